#!/bin/bash
# perm selector in a VGPR (FL_VSEL at d = 64) vs the compiler's SGPR: microbenchmark, parity subset, A/B
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/vsel gpurun_out/ubench
timeout -k 10 120 ./tools/ubench/perm_sgpr > gpurun_out/ubench/perm_sgpr.txt 2>&1 || exit 1
cat gpurun_out/ubench/perm_sgpr.txt
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/vsel/libqmha.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8 and not 128 and not 32" > gpurun_out/vsel/tests.log 2>&1; rc=$?
echo "alt tests rc=$rc: $(tail -1 gpurun_out/vsel/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh vsel/ab_b "--steps 20 --warmup 20 --no-refconfig" default=default vsel=vsel || exit $?
bash tools/ab_env.sh vsel/ab_pt "--variant fa_tc_int8_pt --steps 20 --warmup 20 --no-refconfig" default=default vsel=vsel
