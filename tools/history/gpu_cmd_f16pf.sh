#!/bin/bash
# fp16 main kernel at 8 waves: next tile's Q@K^T issued before the softmax (F16_PREFETCH) vs default
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/f16pf
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/f16pf/libqmha.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "v1a" > gpurun_out/f16pf/tests.log 2>&1; rc=$?
echo "alt tests rc=$rc: $(tail -1 gpurun_out/f16pf/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh f16pf/ab "--variant fa_tc_v1a --steps 20 --warmup 20" default=default prefetch=f16pf
