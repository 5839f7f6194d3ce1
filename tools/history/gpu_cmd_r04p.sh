#!/bin/bash
# r04p: HEAD with the single-read per-tensor pre-pass -- GPU suite + smoke, batch independence of both
# int8 variants, the HEAD bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_cmd_tests.sh r04p || exit $?
O=gpurun_out/r04p
timeout -k 10 300 python tools/det_check.py --rounds 2 > $O/det.log 2>&1; rc=$?; grep -v amdgpu.ids $O/det.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 700 $O/bench.json; echo
