#!/bin/bash
# r04m: determinism / batch independence of the int8 variants, shipped library and alt_lib/pt1
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 300 python tools/det_check.py > $O/det_default.log 2>&1; rc=$?; cat $O/det_default.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
env QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/pt1/libqmha.so timeout -k 10 300 python tools/det_check.py --variants fa_tc_int8_pt > $O/det_pt1.log 2>&1; rc=$?; cat $O/det_pt1.log | grep -v amdgpu.ids; exit $rc
