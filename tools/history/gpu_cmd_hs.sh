#!/bin/bash
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/hs
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "other_head" > gpurun_out/hs/tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed|max\|gpu" gpurun_out/hs/tests.log | tail -12; exit $rc
