#!/bin/bash
# r05o: the per-block O fold as packed fp32 fmas (QMHA_FOLD_PK=1, alt_lib/pk) -- bit identity against the
# shipped build at seven shapes, then same-box alternating A/B of the calling patterns
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05o; mkdir -p $O
ALT=$PWD/quantizedmha_amd/alt_lib/pk/libqmha.so
timeout -k 10 200 python tools/r05/cmp_libs.py $PWD/quantizedmha_amd/lib/libqmha.so $ALT > $O/cmp.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/cmp.txt; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for L in default pk; do
    if [ $L = default ]; then LP=""; else LP=$ALT; fi
    QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,async1,ref > $O/probe_${L}_r$r.txt 2>&1 || { tail -5 $O/probe_${L}_r$r.txt; exit 1; }
    echo "$L r$r: $(tail -1 $O/probe_${L}_r$r.txt)"
  done
done
