#!/bin/bash
# r06 PMC passes at HEAD: HBM traffic (FETCH_SIZE x2 / WRITE_SIZE, separate passes) and the SQ passes for the
# int8 per-block, per-tensor and fp16 main kernels at the C4 shape.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06pmc}
for v in fa_tc_int8_b fa_tc_int8_pt fa_tc_v1a; do
  bash tools/pmc_traffic.sh $TAG/traffic_$v r06 $v 16 16 4096 64 > /tmp/pmc_$v.log 2>&1 || { tail -20 /tmp/pmc_$v.log; exit 1; }
  tail -3 gpurun_out/$TAG/traffic_$v/summary.txt
  BENCH_ARGS="--variant $v" bash tools/pmc_sq.sh $TAG/sq_$v > /tmp/sq_$v.log 2>&1 || { tail -20 /tmp/sq_$v.log; exit 1; }
  grep -E "mfma_busy|valu_insts_per_wave" gpurun_out/$TAG/sq_$v/summary.txt | head -4
done
exit 0
