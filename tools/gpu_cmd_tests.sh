#!/bin/bash
# GPU parity suite + smoke on the box (round 4): logs under gpurun_out/<tag>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r04t}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" $O/tests.log | tail -3
if [ $rc -ne 0 ]; then grep -B5 -A40 "FAILED\|Error" $O/tests.log | head -80; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
exit $rc
