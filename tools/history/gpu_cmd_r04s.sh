#!/bin/bash
# r04s: the per-tensor pre-pass's forced-fallback test plus the per-tensor / NaN / graph subset
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "pt or per_tensor or nan or graph" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; grep "fallback" $O/tests.log | head; exit $rc
