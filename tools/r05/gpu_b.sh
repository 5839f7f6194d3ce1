#!/bin/bash
# r05b: why the fused int8 kernel is slower -- kernel-trace of the calling patterns in both modes, then SQ
# counters of the fused and the two-launch C4 call (batched burst only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05b; mkdir -p $O
for m in 0 1; do
  QMHA_FUSED=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt$m -o run --output-format csv -- python3 tools/probe_calls.py --reps 5 --bursts batched,async1 > $O/kt$m.log 2>&1 || { tail -20 $O/kt$m.log; exit 1; }
  find $O/kt$m -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_m$m.csv \;
  find $O/kt$m -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace_m$m.csv \;
  rm -rf $O/kt$m
done
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM"; do
  i=$((i+1))
  for m in 0 1; do
    QMHA_FUSED=$m timeout -k 10 120 rocprofv3 --pmc $ctr -d $O/pmc_m$m/pmc$i -o run --output-format csv -- python3 tools/probe_calls.py --reps 3 --bursts batched > $O/pmc_m${m}_$i.log 2>&1 || { tail -20 $O/pmc_m${m}_$i.log; exit 1; }
  done
done
for m in 0 1; do python3 tools/pmc_summary.py $O/pmc_m$m --kernel qmha > $O/sq_summary_m$m.txt 2>&1; cat $O/sq_summary_m$m.txt | head -40; done
