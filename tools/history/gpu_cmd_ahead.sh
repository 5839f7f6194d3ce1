#!/bin/bash
# per-tensor kernel: MFMA operands read 3 slots ahead (QMHA_PT_AHEAD=3) vs 2
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/ahead
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/ptahead3/libqmha.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8_pt or per_tensor" > gpurun_out/ahead/tests.log 2>&1; rc=$?
echo "alt tests rc=$rc: $(tail -1 gpurun_out/ahead/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh ahead/ab64 "--variant fa_tc_int8_pt --steps 20 --warmup 20 --no-refconfig" two=default three=ptahead3 || exit $?
bash tools/ab_env.sh ahead/ab128 "--variant fa_tc_int8_pt --B 16 --H 8 --N 4096 --d 128 --steps 20 --warmup 20 --no-refconfig" two=default three=ptahead3
