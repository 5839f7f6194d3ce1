#!/bin/bash
# r04i: VERDICT r03 item 2 -- per-block int8 with P@V accumulated in the MFMA accumulator (f16 P'
# operand carrying the tile scale; alt_lib/f16acc): parity at C4 and on the edge cases, same-box
# alternating timing A/B against the shipped library, SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04i; mkdir -p $O
ALT=$PWD/quantizedmha_amd/alt_lib/f16acc/libqmha.so
env QMHA_LIB_PATH=$ALT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
    -k "full_baseline_config_all_heads or c5_global or growing or large_first or underflow or variant_vs_oracle_random or reference_own_config_int8" > $O/tests_f16acc.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_f16acc.log | tail -2; [ $rc -le 1 ] || exit $rc
for rep in 1 2 3; do
  for lib in default f16acc; do
    if [ "$lib" = default ]; then LP=""; else LP=$ALT; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1 > $O/probe_${lib}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -5 $O/probe_${lib}_$rep.log; exit $rc; }
    echo "$lib rep $rep: $(tail -1 $O/probe_${lib}_$rep.log)"
  done
done | tee $O/ab_summary.txt
QMHA_LIB_PATH=$ALT BENCH_ARGS="--no-solve-calls" bash tools/pmc_sq.sh r04i_sq || exit $?
