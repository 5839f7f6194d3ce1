#!/bin/bash
# scalar fa: explicit op_sel-broadcast v_pk_fma_f32 (default) vs the compiler's packing (alt fanopk)
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/fapk
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "fa] or fa-" > gpurun_out/fapk/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/fapk/tests.log)"; grep "^fa " gpurun_out/fapk/tests.log | head -20; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh fapk/ab "--variant fa --B 8 --H 8 --N 1024 --d 64 --steps 50 --warmup 30 --no-refconfig" pkasm=default compiler=fanopk || exit $?
bash tools/ab_env.sh fapk/ab32 "--variant fa --B 8 --H 16 --N 1024 --d 32 --steps 50 --warmup 30 --no-refconfig" pkasm=default compiler=fanopk
