#!/bin/bash
# r04g: HEAD GPU suite + smoke with issue-priority fairness for few-round grids, then a same-box
# alternating A/B against the previous library (alt_lib/base): batched C4, one sequence per call
# (async and blocking solve()), the reference's shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
bash tools/gpu_cmd_tests.sh r04g || exit $?
O=gpurun_out/r04g; mkdir -p $O
for rep in 1 2 3; do
  for lib in base default; do
    if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1,solve,ref > $O/probe_${lib}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -5 $O/probe_${lib}_$rep.log; exit $rc; }
    echo "$lib rep $rep: $(tail -1 $O/probe_${lib}_$rep.log)"
  done
done | tee $O/ab_summary.txt
