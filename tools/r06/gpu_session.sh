#!/bin/bash
# r06 evidence session on the current tree: GPU parity suite (incl. the concurrent-caller test), smoke, the
# default bench line (clock probe, power cap, isa_sha16), the same bench under rocprofv3 --kernel-trace
# --stats, and the timed-window averages of the main kernels.  Stops at the first failure / timeout.
# usage: bash tools/r06/gpu_session.sh <tag> [--no-tests]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06}; OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -rfE > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
  if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR|Timeout" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc: $(tail -1 $OUT/smoke.log)"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "import json; j=json.load(open('$OUT/bench.json')); print({k: j.get(k) for k in ('value','ms_per_step','clock_ghz','cycles_per_tile','power_cap_w','isa_sha16')}, j['roofline']['main_kernel_ms'], j['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $OUT/trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/trace.log; exit $rc; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/trace -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
rm -rf $OUT/trace
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi65E" 30 50 > $OUT/trace_window.txt
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_int8_pt_v3_kernelILi64ELi8ELi2ELb0E" 2 25 >> $OUT/trace_window.txt
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_f16_v3_kernelILi64" 10 25 >> $OUT/trace_window.txt
cat $OUT/trace_window.txt
exit 0
