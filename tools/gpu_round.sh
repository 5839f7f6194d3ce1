#!/bin/bash
# One GPU session: parity tests, smoke, a short bench.  Stops at the first GPU crash
# (exit codes other than 0 / 1 from pytest), per the pool's rules.
#   PYTEST_ARGS  extra pytest arguments (e.g. "-k int8" or "-x")
#   BENCH_ARGS   extra bench.py arguments;  TAG  output sub-directory of gpurun_out/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-round}; mkdir -p $OUT
export PYTHONUNBUFFERED=1
rocm-smi --showproductname > $OUT/smi.txt 2>&1 || true
timeout -k 10 1200 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfE ${PYTEST_ARGS} > $OUT/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 $OUT/gpu_tests.log | grep -v "^tests/" | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "GPU step crashed/timed out ($rc); stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc2=$?
echo "smoke rc=$rc2"; tail -3 $OUT/smoke.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
[ -n "$NO_BENCH" ] && exit $(( rc | rc2 ))
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc3=$?
echo "bench rc=$rc3"; head -c 3000 $OUT/bench.json; tail -3 $OUT/bench.err
exit $(( rc | rc2 | rc3 ))
