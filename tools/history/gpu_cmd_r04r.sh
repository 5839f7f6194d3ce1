#!/bin/bash
# r04r: single-read per-tensor pre-pass, workgroup size A/B (12 waves shipped; 6 = two workgroups per
# CU; 8 = one workgroup of two waves per SIMD), same box alternating, after a parity subset per build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04r; mkdir -p $O
for lib in ptw6 ptw8; do
  env QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "pt_full_config or pt_quantised or nan or graph" > $O/tests_$lib.log 2>&1
  rc=$?; echo "$lib: $(grep -E 'passed|failed' $O/tests_$lib.log | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_run.sh r04r/ab fa_tc_int8_pt "default ptw6 ptw8" 3 || exit $?
