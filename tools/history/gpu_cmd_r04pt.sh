cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp PYTHONUNBUFFERED=1; mkdir -p gpurun_out/r04pt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "pt or per_tensor or nan" > gpurun_out/r04pt/tests.log 2>&1; rc=$?; tail -2 gpurun_out/r04pt/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_run.sh r04pt/ab fa_tc_int8_pt "pt2pass default ptfwd pt2cu ptw8" 3
