#!/bin/bash
# r03m: fp16 workgroup-size A/B (8-wave default vs 4-wave alt build) at d = 32 / 64 / 128
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/wg2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "fa_tc_v1a or c3_fp16 or fp16" > gpurun_out/wg2/tests_f16.log 2>&1; rc=$?; echo "fp16 tests rc=$rc $(tail -1 gpurun_out/wg2/tests_f16.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh wg2/d64 "--variant fa_tc_v1a --no-refconfig --steps 20 --warmup 5" w8=default w4=f16w4 w8sg4=abl:QMHA_F16_CFG=484 || exit $?
bash tools/ab_env.sh wg2/d32 "--variant fa_tc_v1a --no-refconfig --steps 20 --warmup 5 --H 32 --d 32" w8=default w4=f16w4 || exit $?
bash tools/ab_env.sh wg2/d128 "--variant fa_tc_v1a --no-refconfig --steps 20 --warmup 5 --H 8 --d 128" w8=default w4=f16w4 || exit $?
