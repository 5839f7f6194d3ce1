#!/bin/bash
# r06: the full GPU suite on the current tree, then a per-tensor-only parity sweep (400 shapes) against the
# base-2 oracle.  Stops at the first failure / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06t}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rfE > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $O/gpu_tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Timeout" $O/gpu_tests.log | head -20; grep -E "^E  " $O/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 400 python tools/r05/sweep.py --n 400 --seed 14 --variants fa_tc_int8_pt > $O/sweep_pt.log 2>&1; rc=$?; tail -1 $O/sweep_pt.log
exit $rc
