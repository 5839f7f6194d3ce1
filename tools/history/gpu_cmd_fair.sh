#!/bin/bash
# FL_FAIR (issue priority falls with sweep progress) vs default: parity subset, A/B, timelines
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/fair
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/fair/libqmha.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -k "int8 and not dump and not debug" > gpurun_out/fair/tests.log 2>&1; rc=$?
echo "fair tests rc=$rc: $(tail -1 gpurun_out/fair/tests.log)"; [ $rc -ne 0 ] && exit $rc
bash tools/ab_env.sh fair/ab_b "--steps 20 --warmup 20" default=default fair=fair || exit $?
bash tools/ab_env.sh fair/ab_pt "--variant fa_tc_int8_pt --steps 20 --warmup 20" default=default fair=fair || exit $?
export QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/fairtl/libqmha.so
for args in "fa_tc_int8_b 1 32 8192 32" "fa_tc_int8_b 16 16 4096 64"; do
  timeout -k 10 120 python tools/timeline.py $args > gpurun_out/fair/tl_$(echo $args | tr ' ' '_').txt 2>&1 || exit 1
  head -5 gpurun_out/fair/tl_$(echo $args | tr ' ' '_').txt; tail -1 gpurun_out/fair/tl_$(echo $args | tr ' ' '_').txt
done
