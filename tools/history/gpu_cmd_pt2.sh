#!/bin/bash
# per-tensor mode: parity subset on the default build, then A/B of the chunked pre-pass
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/pt2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8_pt" > gpurun_out/pt2/tests.log 2>&1; rc=$?
echo "pt tests rc=$rc: $(tail -1 gpurun_out/pt2/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh pt2/ab "--variant fa_tc_int8_pt --steps 20 --warmup 10 --no-refconfig" chunked=default whole=ptnochunk
timeout -k 10 240 python bench.py --variant fa_tc_int8_pt --steps 20 --warmup 10 --no-siblings --no-cpu-baseline > gpurun_out/pt2/pt_refcfg.json 2> gpurun_out/pt2/pt_refcfg.err
