#!/bin/bash
# per-tensor d = 128: Q@K^T steps interleaved with P@V (QMHA_PT_D128_SCHED=1) vs paired
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/d128b
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/ptd128b/libqmha.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8_pt or per_tensor" > gpurun_out/d128b/tests.log 2>&1; rc=$?
echo "alt tests rc=$rc: $(tail -1 gpurun_out/d128b/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh d128b/ab "--variant fa_tc_int8_pt --B 16 --H 8 --N 4096 --d 128 --steps 20 --warmup 20 --no-refconfig" paired=default split=ptd128b
