#!/bin/bash
# r05h: fused int8 with single-wave flag polling (the other waves at the barrier) and the production as a
# non-inlined call -- fused tests, then same-box alternating A/B against the two launches
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_zfused.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_fused.log 2>&1
rc=$?; tail -1 $O/tests_fused.log; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" $O/tests_fused.log | head -30; exit $rc; }
for r in 1 2 3; do
  for m in 0 1; do
    QMHA_FUSED=$m timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1 > $O/probe_m${m}_r$r.txt 2>&1 || { tail -5 $O/probe_m${m}_r$r.txt; exit 1; }
    echo "int8 fused=$m r$r: $(tail -1 $O/probe_m${m}_r$r.txt)"
  done
done
