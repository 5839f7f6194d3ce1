#!/bin/bash
# r06: extended random-shape parity sweep at HEAD (the lazy-base fp16 and per-tensor kernels): 400 shapes, a
# new seed, four variants against the oracle, fa_tc_v1a also against its own lazy contract.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06sweep}; mkdir -p $O
timeout -k 10 500 python tools/r05/sweep.py --n 400 --seed ${2:-13} > $O/sweep_head.log 2>&1; rc=$?; tail -1 $O/sweep_head.log
exit $rc
