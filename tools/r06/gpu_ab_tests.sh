#!/bin/bash
# r06: a parity subset (pytest -k "$2"), then the same-box alternating A/B of alt_lib/$3 vs the current build.
# usage: bash tools/r06/gpu_ab_tests.sh <tag> <pytest -k expr> <base-alt-lib> <variants> [extra shapes...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; K=$2; shift 2; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rfE -k "$K" > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Timeout" $OUT/tests.log | head -20; grep -E "max\|gpu-oracle" $OUT/tests.log | tail -40; exit $rc; fi
grep -E "fa_tc_v1a +max" $OUT/tests.log | sort -k3 -g | tail -8
bash tools/r06/gpu_ab.sh $TAG "$@"
