cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out/r04f16p
for lib in f16p f16pj; do
  env QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "fa_tc_v1a" > gpurun_out/r04f16p/tests_$lib.log 2>&1; rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/r04f16p/tests_$lib.log)"; [ $rc -eq 0 ] || { grep -A30 FAIL gpurun_out/r04f16p/tests_$lib.log | head -60; exit $rc; }
done
bash tools/ab_run.sh r04f16p/ab fa_tc_v1a "default f16p f16pj" 3
bash tools/ab_run.sh r04f16p/ab32 fa_tc_v1a "default f16p f16pj" 2 "--d 32 --H 32"
