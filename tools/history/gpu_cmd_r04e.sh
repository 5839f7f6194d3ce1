#!/bin/bash
# r04e: SQ counters of the fa_tc_int8_b main kernel at one C4 sequence per launch (2 waves/SIMD)
# against the batched C4 launch (3 waves/SIMD): where the under-filled grid loses its time
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
BENCH_ARGS="--B 1 --no-solve-calls" bash tools/pmc_sq.sh r04e_b1 || exit $?
BENCH_ARGS="--no-solve-calls" bash tools/pmc_sq.sh r04e_b16 || exit $?
