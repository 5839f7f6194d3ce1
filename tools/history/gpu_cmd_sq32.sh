#!/bin/bash
# SQ counters at the reference's shape (B1 H32 N8192 d32): per-tensor vs per-block main kernel
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1
BENCH_ARGS="--variant fa_tc_int8_pt --B 1 --H 32 --N 8192 --d 32 --no-solve-calls" bash tools/pmc_sq.sh sq32/pt || exit $?
BENCH_ARGS="--variant fa_tc_int8_b --B 1 --H 32 --N 8192 --d 32 --no-solve-calls" bash tools/pmc_sq.sh sq32/pb || exit $?
