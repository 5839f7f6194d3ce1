#!/bin/bash
# r05u: extended random-shape parity sweeps at the final HEAD (default build, a new seed) and on the
# per-tensor int8 P@V A/B build (alt_lib/pt8, the per-tensor variant only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r05u}; mkdir -p $O
timeout -k 10 400 python tools/r05/sweep.py --n 400 --seed 11 > $O/sweep_head.log 2>&1; rc=$?; tail -1 $O/sweep_head.log; [ $rc -gt 1 ] && exit $rc
QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/pt8/libqmha.so timeout -k 10 400 python tools/r05/sweep.py --n 300 --seed 12 --variants fa_tc_int8_pt > $O/sweep_pt8.log 2>&1; rc=$?; tail -1 $O/sweep_pt8.log
exit 0
