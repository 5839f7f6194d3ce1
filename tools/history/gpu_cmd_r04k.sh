#!/bin/bash
# r04k: HEAD PMC passes for bench.py's roofline.traffic / mfma_busy (FETCH_SIZE, WRITE_SIZE per
# variant at C4; SQ counters of the int8 main kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in fa_tc_int8_b fa_tc_int8_pt fa_tc_v1a; do
  bash tools/pmc_traffic.sh r04k_$v r04 $v 16 16 4096 64 || exit $?
done
for v in fa_tc_int8_b fa_tc_int8_pt; do
  BENCH_ARGS="--no-solve-calls --variant $v" bash tools/pmc_sq.sh r04k_sq_$v > /dev/null || exit $?
  python3 tools/pmc_summary.py gpurun_out/r04k_sq_$v --kernel qmha --json-out gpurun_out/r04k_sq_$v/pmc_sq_$v.json --shape 16 16 4096 64 > gpurun_out/r04k_sq_$v/summary.txt || exit $?
done
ls gpurun_out/r04k_*/*.json
