#!/bin/bash
# One evidence session on HEAD: GPU parity suite, smoke, the default bench line (siblings, CPU
# baseline), then the same bench under rocprofv3 --kernel-trace --stats and the timed-window
# averages of the int8 and fp16 main kernels.  Stops at the first GPU crash / timeout.
# usage: bash tools/gpu_final.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-final}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -rfE > $OUT/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then tail -30 $OUT/gpu_tests.log; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc: $(tail -1 $OUT/smoke.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $OUT/trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"; [ $rc -ne 0 ] && { tail -20 $OUT/trace.log; exit $rc; }
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/trace -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi65E" 30 50 > $OUT/trace_window.txt
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi1048641E" 2 25 >> $OUT/trace_window.txt
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_f16_v2_kernelILi64" 10 25 >> $OUT/trace_window.txt
cat $OUT/trace_window.txt
exit 0
