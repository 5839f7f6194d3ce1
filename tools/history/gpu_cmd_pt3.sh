#!/bin/bash
# per-tensor mode at d = 32: 4-wave register budget (default) vs 3 (alt ptd32lb3), at the reference's shape
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/pt3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8_pt" > gpurun_out/pt3/tests.log 2>&1; rc=$?
echo "pt tests rc=$rc: $(tail -1 gpurun_out/pt3/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh pt3/ab "--variant fa_tc_int8_pt --steps 10 --warmup 10" lb4=default lb3=ptd32lb3
