#!/bin/bash
# SQ-level PMC passes on the default bench (int8 main kernel): clock, issue, waits, MFMA.
# usage: bash tools/pmc_sq.sh <tag>     (env BENCH_ARGS adds bench flags, QMHA_* envs pass through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-sq}; OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-siblings --no-refconfig ${BENCH_ARGS} > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/pmc$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT --kernel qmha > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
