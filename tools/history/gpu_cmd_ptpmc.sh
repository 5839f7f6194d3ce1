#!/bin/bash
# per-tensor mode at C4: HBM traffic passes and SQ counters
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1
bash tools/pmc_traffic.sh ptpmc/traffic r03 fa_tc_int8_pt 16 16 4096 64 || exit $?
BENCH_ARGS="--variant fa_tc_int8_pt --no-solve-calls" bash tools/pmc_sq.sh ptpmc/sq || exit $?
