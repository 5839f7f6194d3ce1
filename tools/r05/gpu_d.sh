#!/bin/bash
# r05d: fused int8 with the fast producer -- bit-identity tests, then same-box alternating A/B: two launches,
# fused (fast quantiser), fused with the exact quantiser for every group (ablate bit 3 = the r04 producer)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_zfused.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_fused.log 2>&1
rc=$?; tail -1 $O/tests_fused.log; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" $O/tests_fused.log | head -30; exit $rc; }
for r in 1 2 3; do
  for cfg in "0 0" "1 0" "1 8"; do
    set -- $cfg
    QMHA_FUSED=$1 QMHA_FUSED_ABLATE=$2 timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1,solve > $O/probe_f$1_a$2_r$r.txt 2>&1 || { tail -5 $O/probe_f$1_a$2_r$r.txt; exit 1; }
    echo "fused=$1 ablate=$2 r$r: $(tail -1 $O/probe_f$1_a$2_r$r.txt)"
  done
done
