#!/bin/bash
# fused int8 path: bit-identity test, int8 parity tests, then bench fused 0/1 alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-ab_fused}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "fused" > $OUT/tests_fused.log 2>&1
rc=$?; echo "fused tests rc=$rc: $(tail -1 $OUT/tests_fused.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "int8 or all_ones" > $OUT/tests_int8.log 2>&1
rc=$?; echo "int8 tests rc=$rc: $(tail -1 $OUT/tests_int8.log)"; [ $rc -ne 0 ] && exit $rc
for f in 0 1 0 1; do
  timeout -k 10 180 python bench.py --int8-fused $f --no-siblings --no-cpu-baseline --no-refconfig --no-solve-calls > $OUT/bench_f$f.json 2> $OUT/bench_f$f.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench rc=$rc"; tail -3 $OUT/bench_f$f.err; exit $rc; }
  python -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print('fused', sys.argv[2], j['ms_per_step'], 'main', r['main_kernel_ms'], 'pre', r['prepass_ms'])" $OUT/bench_f$f.json $f
done
