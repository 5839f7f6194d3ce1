#!/bin/bash
# first-round vs steady-state workgroup durations (production schedule + timeline probe)
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/tl2
export QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/tl/libqmha.so
for args in "fa_tc_int8_b 1 32 8192 32" "fa_tc_int8_b 4 32 8192 32" "fa_tc_int8_b 16 16 4096 64" "fa_tc_int8_pt 1 32 8192 32"; do
  timeout -k 10 120 python tools/timeline.py $args > gpurun_out/tl2/tl_$(echo $args | tr ' ' '_').txt 2>&1 || exit 1
  head -5 gpurun_out/tl2/tl_$(echo $args | tr ' ' '_').txt
done
