#!/bin/bash
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/maxn
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "maximum" > gpurun_out/maxn/tests.log 2>&1; rc=$?
tail -15 gpurun_out/maxn/tests.log; exit $rc
