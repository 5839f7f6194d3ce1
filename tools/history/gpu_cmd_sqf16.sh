#!/bin/bash
# SQ counters of the fp16 main kernel at HEAD (8-wave workgroups) and its HBM traffic
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1
BENCH_ARGS="--variant fa_tc_v1a --no-solve-calls" bash tools/pmc_sq.sh sqf16 || exit $?
bash tools/pmc_traffic.sh trf16 r03 fa_tc_v1a 16 16 4096 64
