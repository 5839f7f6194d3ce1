#!/bin/bash
# Ablation sweep of the int8 main kernel (needs a QMHA_EXTRA_FLAGS=-DQMHA_ABLATION build).
# usage: bash tools/ablate.sh <tag> "<abl values>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-abl}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for a in $2; do
  QMHA_INT8_ABL=$a timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > $OUT/abl_$a.json 2>$OUT/abl_$a.err
  rc=$?; [ $rc -ne 0 ] && { echo "abl $a rc=$rc"; tail -3 $OUT/abl_$a.err; exit $rc; }
  python - "$a" $OUT/abl_$a.json <<'PY'
import json,sys; j=json.load(open(sys.argv[2])); print("abl", sys.argv[1], j["ms_per_step"], j["roofline"]["main_kernel_ms"])
PY
done
