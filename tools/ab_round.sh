#!/bin/bash
# GPU A/B round: parity tests on the default build, then bench.py A/B (default vs alt_lib/<names>)
# for the int8 and fp16 variants.  usage: bash tools/ab_round.sh <tag> "<alt names>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/gpu_tests.log; exit $rc; fi
echo "int8:"; bash tools/ab_bench.sh $TAG/i8 "$2" "" || exit $?
echo "fp16:"; bash tools/ab_bench.sh $TAG/f16 "$2" "--variant fa_tc_v1a --no-refconfig" || exit $?
