#!/bin/bash
# timing perturbations of the int8 d=64 main kernel: default vs no-MFMA vs no-exp builds
# (QMHA_ABLATION-style alt libs, results wrong by design), alternating, full warm-up
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-perturb}; mkdir -p $OUT
for lib in ${LIBS:-default nomfma noexp default nomfma noexp}; do
  if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
  QMHA_LIB_PATH=$LP timeout -k 10 180 python bench.py --no-siblings --no-cpu-baseline --no-refconfig --no-solve-calls > $OUT/bench_$lib.json 2> $OUT/bench_$lib.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $lib rc=$rc"; tail -3 $OUT/bench_$lib.err; exit $rc; }
  python -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print(sys.argv[2], j['ms_per_step'], 'main', r['main_kernel_ms'])" $OUT/bench_$lib.json $lib
done
