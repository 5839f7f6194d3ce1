#!/bin/bash
# r06: the lazy-base staircase tests, and where the two per-block sweep failures of seed 13 (shapes 188, 288:
# flip fraction only) put their elements above 5e-5 (tools/r05/sweep.py --only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06chk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "staircase" -v --timeout 120 --timeout-method thread -rfE > $O/staircase.log 2>&1
rc=$?; echo "staircase rc=$rc: $(tail -1 $O/staircase.log)"; [ $rc -ne 0 ] && { tail -30 $O/staircase.log; exit $rc; }
for i in 188 288; do
  timeout -k 10 300 python tools/r05/sweep.py --n 400 --seed 13 --only $i --variants fa_tc_int8_b > $O/only_$i.log 2>&1; rc=$?
  echo "only $i rc=$rc"; [ $rc -gt 1 ] && exit $rc
done
exit 0
