#!/bin/bash
# HEAD check: full GPU parity suite and smoke (no bench)
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/head
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/head/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc: $(tail -1 gpurun_out/head/gpu_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/head/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc: $(tail -1 gpurun_out/head/smoke.log)"; exit $rc
