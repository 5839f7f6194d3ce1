#!/bin/bash
# fp32 sibling A/B at C2 (B8 H8 N1024 d64): parity tests of `fa` on the default build, then
# bench default vs alt_lib builds, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-ab_f32}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
for lib in default $2 default $2; do
  if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
  QMHA_LIB_PATH=$LP timeout -k 10 120 python bench.py --variant fa --B 8 --H 8 --N 1024 --no-siblings --no-cpu-baseline --no-refconfig --no-solve-calls > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $lib rc=$rc"; tail -3 $OUT/bench_$lib.err; exit $rc; }
  python -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print(sys.argv[2], j['ms_per_step'], 'main', r['main_kernel_ms'], 'frac', r['frac'])" $OUT/bench_$lib.json $lib
done
