#!/bin/bash
# Parity subset, then bench at several QMHA_OVERLAP_CHUNKS values for the int8 and fp16 paths.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-ovl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/tests.log; exit $rc; fi
for v in fa_tc_int8_b fa_tc_v1a; do
  for c in ${2:-1 2 4 8}; do
    QMHA_OVERLAP_CHUNKS=$c timeout -k 10 120 python bench.py --variant $v --steps 20 --warmup 5 --no-siblings --no-cpu-baseline > $OUT/bench_${v}_$c.json 2>$OUT/bench_${v}_$c.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $v $c rc=$rc"; tail -3 $OUT/bench_${v}_$c.err; exit $rc; }
    python - "$v chunks=$c" $OUT/bench_${v}_$c.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); r=j["roofline"]; print("   ", sys.argv[1], "ms", j["ms_per_step"], "value", j["value"], "main", r["main_kernel_ms"], "pre", r["prepass_ms"])
PY
  done
done
