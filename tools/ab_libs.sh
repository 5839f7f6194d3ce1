#!/bin/bash
# A/B: bench QMHA_INT8_CFG codes against several builds of libqmha.so (quantizedmha_amd/alt_lib/*).
# usage: bash tools/ab_libs.sh <tag> "<lib names: default or alt_lib dir names>" "<cfg codes>" [parity]
# env: VARIANT (default fa_tc_int8_b), CFGVAR (default QMHA_INT8_CFG), TESTK (pytest -k filter)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
VARIANT=${VARIANT:-fa_tc_int8_b}; CFGVAR=${CFGVAR:-QMHA_INT8_CFG}; TESTK=${TESTK:-int8 or all_ones}
for lib in $2; do
  if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
  for c in $3; do
    if [ -n "$4" ]; then
      env QMHA_LIB_PATH=$LP $CFGVAR=$c timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "$TESTK" > $OUT/tests_${lib}_$c.log 2>&1
      rc=$?; echo "$lib $c tests rc=$rc: $(tail -1 $OUT/tests_${lib}_$c.log)"
      if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    fi
    env QMHA_LIB_PATH=$LP $CFGVAR=$c timeout -k 10 120 python bench.py --variant $VARIANT --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > $OUT/bench_${lib}_$c.json 2>$OUT/bench_${lib}_$c.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $lib $c rc=$rc"; tail -3 $OUT/bench_${lib}_$c.err; exit $rc; }
    python - "$lib $c" $OUT/bench_${lib}_$c.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); print("   ", sys.argv[1], j["ms_per_step"], "main", j["roofline"]["main_kernel_ms"], "frac", j["roofline"]["frac"])
PY
  done
done
