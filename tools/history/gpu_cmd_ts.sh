#!/bin/bash
# r03n: int8 FL_TSHADOW (MFMA shadows filled with transcendental / quarter-rate work) parity + A/B
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/ts
for c in 9300 9200; do
  QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/abl/libqmha.so QMHA_INT8_CFG=$c timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "int8 or all_ones or full_baseline or reference_own" > gpurun_out/ts/tests_$c.log 2>&1; rc=$?
  echo "cfg $c rc=$rc $(tail -1 gpurun_out/ts/tests_$c.log)"; [ $rc -ne 0 ] && exit $rc
done
bash tools/ab_env.sh ts/d64 "--steps 20 --warmup 10 --no-refconfig" default=default ts=abl:QMHA_INT8_CFG=9300 acc1=abl:QMHA_INT8_CFG=9200
