#!/bin/bash
# r04d: head-ahead schedule (FL_HA) -- bit-identity tests, then a same-box alternating A/B of the
# fa_tc_int8_b main-kernel schedules (1 = three-wave, 2 = head-ahead) batched, one sequence per call,
# and the reference's own shape (B = 1, 2, 4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "head_ahead or production_qk_int32_bitexact or deterministic or growing or large_first or underflow" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tests.log | head -60; exit $rc; }
for rep in 1 2 3; do
  for s in 1 2; do
    env QMHA_SCHED=$s timeout -k 10 120 python tools/probe_calls.py --reps 10 --bursts batched,async1,ref > $O/probe_s${s}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "sched $s rc=$rc"; tail -5 $O/probe_s${s}_$rep.log; exit $rc; }
    echo "sched $s rep $rep: $(tail -1 $O/probe_s${s}_$rep.log)"
  done
done | tee $O/ab_summary.txt
