#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Stops at the first GPU crash
# (exit codes other than 0 / 1 from pytest), per the pool's rules.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU step crashed/timed out ($rc); stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?
echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc3=$?
echo "bench rc=$rc3"; tail -3 gpurun_out/bench.log
exit $(( rc | rc2 | rc3 ))
