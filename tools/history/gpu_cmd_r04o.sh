#!/bin/bash
# r04o: single-read per-tensor pre-pass with XCD-local slice parts (alt_lib/pt1: 32 KiB per wave,
# alt_lib/pt1s: 16 KiB per wave) -- batch independence, parity subset, A/B against the shipped pre-pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04o; mkdir -p $O
for lib in pt1w12 pt1k48; do
  ALT=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so
  env QMHA_LIB_PATH=$ALT timeout -k 10 300 python tools/det_check.py --variants fa_tc_int8_pt --rounds 2 > $O/det_$lib.log 2>&1
  rc=$?; grep -v amdgpu.ids $O/det_$lib.log; [ $rc -eq 0 ] || exit $rc
  env QMHA_LIB_PATH=$ALT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "pt or per_tensor or nan" > $O/tests_$lib.log 2>&1
  rc=$?; echo "$lib: $(grep -E 'passed|failed' $O/tests_$lib.log | tail -1)"; [ $rc -eq 0 ] || { grep -B3 -A25 "FAILED\|Error" $O/tests_$lib.log | head -60; exit $rc; }
done
bash tools/ab_run.sh r04o/ab fa_tc_int8_pt "default pt1 pt1w12 pt1k48" 3 || exit $?
