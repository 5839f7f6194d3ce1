#!/bin/bash
# r05q: per-tensor int8 P@V on the i8 matrix core into an int32 window (QMHA_INT8_PT_I8PV=1, alt_lib/pt8) --
# the per-tensor GPU parity tests on that build, same-box alternating A/B of the calling patterns, kernel
# traces and SQ counters of both builds' C4 call
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r05s}; mkdir -p $O
ALT=$PWD/quantizedmha_amd/alt_lib/pt8/libqmha.so
QMHA_LIB_PATH=$ALT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "pt" -x -v --timeout 300 --timeout-method thread > $O/tests_pt8.log 2>&1
rc=$?; echo "pt8 tests rc=$rc"; grep -E "passed|failed|error" $O/tests_pt8.log | tail -3
if [ $rc -ne 0 ]; then grep -B5 -A40 "FAILED\|Error" $O/tests_pt8.log | head -80; exit $rc; fi
for r in 1 2 3; do
  for L in default pt8; do
    if [ $L = default ]; then LP=""; else LP=$ALT; fi
    QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --variant fa_tc_int8_pt --reps 10 --bursts batched,async1,ref > $O/probe_${L}_r$r.txt 2>&1 || { tail -5 $O/probe_${L}_r$r.txt; exit 1; }
    echo "$L r$r: $(tail -1 $O/probe_${L}_r$r.txt)"
  done
done
for L in default pt8; do
  if [ $L = default ]; then LP=""; else LP=$ALT; fi
  QMHA_LIB_PATH=$LP timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$L -o run --output-format csv -- python3 tools/probe_calls.py --variant fa_tc_int8_pt --reps 5 --bursts batched > $O/kt_$L.log 2>&1 || { tail -20 $O/kt_$L.log; exit 1; }
  find $O/kt_$L -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$L.csv \;
  rm -rf $O/kt_$L
  grep -h "pipe_kernel\|pt_quant" $O/kernel_stats_$L.csv | cut -d, -f1-4
done
i=0
for ctr in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_COEXEC_CYCLES"; do
  i=$((i+1))
  for L in default pt8; do
    if [ $L = default ]; then LP=""; else LP=$ALT; fi
    QMHA_LIB_PATH=$LP timeout -k 10 120 rocprofv3 --pmc $ctr -d $O/pmc_$L/pmc$i -o run --output-format csv -- python3 tools/probe_calls.py --variant fa_tc_int8_pt --reps 3 --bursts batched > $O/pmc_${L}_$i.log 2>&1 || { tail -20 $O/pmc_${L}_$i.log; exit 1; }
  done
done
for L in default pt8; do python3 tools/pmc_summary.py $O/pmc_$L --kernel qmha > $O/sq_summary_$L.txt 2>&1; grep -A30 "pipe_kernel" $O/sq_summary_$L.txt | head -30; done
