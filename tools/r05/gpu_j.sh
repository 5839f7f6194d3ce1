#!/bin/bash
# r05j: timing ablations (results wrong) for int8 P@V in the per-block kernel: i8pv = one i8 MFMA per d-block
# instead of two f16 ones (the matrix-core saving alone); i8pvf = plus the packed bias-removing O fold it needs
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05j; mkdir -p $O
for r in 1 2 3; do
  for L in default i8pv i8pvf; do
    if [ $L = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$L/libqmha.so; fi
    QMHA_LIB_PATH=$LP timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts batched,ref > $O/probe_${L}_r$r.txt 2>&1 || { tail -5 $O/probe_${L}_r$r.txt; exit 1; }
    echo "$L r$r: $(tail -1 $O/probe_${L}_r$r.txt)"
  done
done
