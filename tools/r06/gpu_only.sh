#!/bin/bash
# r06: where the two per-block sweep failures of seed 13 (shapes 188, 288: flip fraction only) put their
# elements above 5e-5 (tools/r05/sweep.py --only prints the (batch, row, head) rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06only}; mkdir -p $O
for i in 188 288; do
  timeout -k 10 300 python tools/r05/sweep.py --n 400 --seed 13 --only $i --variants fa_tc_int8_b > $O/only_$i.log 2>&1; rc=$?
  echo "only $i rc=$rc"; cat $O/only_$i.log | head -5; [ $rc -gt 1 ] && exit $rc
done
exit 0
