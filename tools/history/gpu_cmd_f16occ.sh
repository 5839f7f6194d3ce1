cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out/r04f16
for lib in f16o5 f16o5w8; do
  env QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fa_tc_v1a and (random or golden or c3 or spike or growing)" > gpurun_out/r04f16/tests_$lib.log 2>&1; rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/r04f16/tests_$lib.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab_run.sh r04f16/ab fa_tc_v1a "default f16o5 f16nov f16o5w8" 3
