#!/bin/bash
# Geometry sweep: bench the int8 / fp16 kernels under each QMHA_*_CFG value.
# usage: bash tools/sweep.sh <tag> "<int8 cfgs>" "<f16 cfgs>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-sweep}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for c in $2; do
  QMHA_INT8_CFG=$c timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > $OUT/int8_$c.json 2>$OUT/int8_$c.err
  rc=$?; [ $rc -ne 0 ] && { echo "int8 $c rc=$rc"; tail -3 $OUT/int8_$c.err; exit $rc; }
  python - "$c" $OUT/int8_$c.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); print("int8", sys.argv[1], j["ms_per_step"], j["roofline"]["main_kernel_ms"], j["roofline"]["frac"])
PY
done
for c in $3; do
  QMHA_F16_CFG=$c timeout -k 10 120 python bench.py --variant fa_tc_v1a --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > $OUT/f16_$c.json 2>$OUT/f16_$c.err
  rc=$?; [ $rc -ne 0 ] && { echo "f16 $c rc=$rc"; tail -3 $OUT/f16_$c.err; exit $rc; }
  python - "$c" $OUT/f16_$c.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); print("f16", sys.argv[1], j["ms_per_step"], j["roofline"]["main_kernel_ms"], j["roofline"]["frac"])
PY
done
