#!/bin/bash
# r05a: the hardened fused int8 bit-identity test (poisoned / other-input scratch, cross-XCD rule on
# multi-round grids), then a same-box alternating A/B of the calling patterns, fused 0 / 1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_zfused.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_fused.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_fused.log | tail -1; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" $O/tests_fused.log | head -30; exit $rc; }
for r in 1 2; do
  for m in 0 1; do
    QMHA_FUSED=$m timeout -k 10 150 python tools/probe_calls.py --reps 10 > $O/probe_m${m}_r$r.txt 2>&1 || { tail -5 $O/probe_m${m}_r$r.txt; exit 1; }
    echo "fused=$m round $r: $(tail -1 $O/probe_m${m}_r$r.txt)"
  done
done
