#!/bin/bash
# r04l: single-read per-tensor pre-pass (alt_lib/pt1: qmha_pt_quant_kernel) -- batch independence
# repeated, its parity tests, a same-box alternating A/B of the fa_tc_int8_pt call against the shipped
# two-pass pre-pass; then the HEAD PMC passes (r04k)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04l; mkdir -p $O
ALT=$PWD/quantizedmha_amd/alt_lib/pt1/libqmha.so
env QMHA_LIB_PATH=$ALT timeout -k 10 300 python tools/det_check.py --variants fa_tc_int8_pt --rounds 4 > $O/det_pt1.log 2>&1
rc=$?; grep -v amdgpu.ids $O/det_pt1.log; [ $rc -eq 0 ] || exit $rc
env QMHA_LIB_PATH=$ALT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "pt or per_tensor or nan" > $O/tests_pt1.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_pt1.log | tail -2; [ $rc -eq 0 ] || { grep -B3 -A25 "FAILED\|Error" $O/tests_pt1.log | head -60; exit $rc; }
bash tools/ab_run.sh r04l/ab fa_tc_int8_pt "default pt1" 3 || exit $?
bash tools/gpu_cmd_r04k.sh
