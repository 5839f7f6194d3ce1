#!/bin/bash
# r04f: issue-priority fairness (s_setprio lowered as the sweep progresses, QMHA_AB_FAIR quarters /
# halves) at one C4 sequence per call (two co-resident workgroups per CU), batched C4, and the
# reference's own shape; same-box alternating A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04f; mkdir -p $O
for rep in 1 2 3; do
  for lib in default fair4 fair2; do
    if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 120 python tools/probe_calls.py --reps 10 --bursts batched,async1,ref > $O/probe_${lib}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -5 $O/probe_${lib}_$rep.log; exit $rc; }
    echo "$lib rep $rep: $(tail -1 $O/probe_${lib}_$rep.log)"
  done
done | tee $O/ab_summary.txt
