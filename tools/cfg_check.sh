#!/bin/bash
# For each QMHA_INT8_CFG code: int8 parity subset, then a short bench.  Stops on a GPU crash.
# usage: bash tools/cfg_check.sh <tag> "<cfg codes>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-cfg}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for c in $2; do
  QMHA_INT8_CFG=$c timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "int8 or all_ones" > $OUT/tests_$c.log 2>&1
  rc=$?; echo "cfg $c tests rc=$rc: $(tail -1 $OUT/tests_$c.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  QMHA_INT8_CFG=$c timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > $OUT/bench_$c.json 2>$OUT/bench_$c.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $c rc=$rc"; tail -3 $OUT/bench_$c.err; exit $rc; }
  python - "$c" $OUT/bench_$c.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); print("   bench", sys.argv[1], j["ms_per_step"], "main", j["roofline"]["main_kernel_ms"], "frac", j["roofline"]["frac"])
PY
done
