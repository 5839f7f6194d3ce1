#!/bin/bash
# r04t: the fused per-block int8 kernel (FL_FUSED): bit-identity vs the two-launch path, the int8 /
# graph / NaN subset, then a same-box alternating A/B of the calling patterns (QMHA_FUSED 0 / 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_zfused.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_fused.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_fused.log | tail -1; [ $rc -ne 0 ] && { tail -30 $O/tests_fused.log; exit $rc; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "int8 or graph or nan or all_ones or reference or c5 or full_baseline" > $O/tests_int8.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_int8.log | tail -1; [ $rc -ne 0 ] && { tail -30 $O/tests_int8.log; exit $rc; }
for r in 1 2; do
  for m in 0 1; do
    QMHA_FUSED=$m timeout -k 10 120 python tools/probe_calls.py --reps 10 > $O/probe_m${m}_r$r.txt 2>&1 || { tail -5 $O/probe_m${m}_r$r.txt; exit 1; }
    echo "fused=$m round $r: $(tail -1 $O/probe_m${m}_r$r.txt)"
  done
done
