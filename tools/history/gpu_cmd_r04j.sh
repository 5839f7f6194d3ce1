#!/bin/bash
# r04j: pre-pass / main-kernel overlap by batch chunks (qmha_set_overlap_chunks) re-measured on the r04
# kernels, int8 and fp16 at C4, same-box alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04j; mkdir -p $O
for rep in 1 2 3; do
  for v in fa_tc_int8_b fa_tc_v1a; do
    for c in 1 2 4; do
      env QMHA_OVERLAP=$c timeout -k 10 120 python tools/probe_calls.py --variant $v --reps 20 --bursts batched > $O/probe_${v}_${c}_$rep.log 2>&1
      rc=$?; [ $rc -ne 0 ] && { echo "$v $c rc=$rc"; tail -5 $O/probe_${v}_${c}_$rep.log; exit $rc; }
      echo "$v chunks $c rep $rep: $(tail -1 $O/probe_${v}_${c}_$rep.log)"
    done
  done
done | tee $O/ab_summary.txt
