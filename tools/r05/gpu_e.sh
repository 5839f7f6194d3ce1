#!/bin/bash
# r05e: 12-wave workgroups for the per-block d = 64 kernel (one workgroup per CU; each LDS-DMA stage shared by
# 12 waves instead of 4) -- bit identity against the shipped 4-wave build, then same-box alternating A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05e; mkdir -p $O
ALT=$PWD/quantizedmha_amd/alt_lib/w12/libqmha.so
timeout -k 10 200 python tools/r05/cmp_libs.py $PWD/quantizedmha_amd/lib/libqmha.so $ALT > $O/cmp.txt 2>&1; rc=$?; cat $O/cmp.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for L in default w12; do
    if [ $L = default ]; then LP=""; else LP=$ALT; fi
    QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1,solve,ref > $O/probe_${L}_r$r.txt 2>&1 || { tail -5 $O/probe_${L}_r$r.txt; exit 1; }
    echo "$L r$r: $(tail -1 $O/probe_${L}_r$r.txt)"
  done
done
