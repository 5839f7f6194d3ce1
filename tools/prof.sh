#!/bin/bash
# Profile session: quick parity, bench, rocprofv3 kernel trace (+ optional PMC pass).
# usage: bash tools/prof.sh <tag> [pmc counters...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
[ -f gpurun_out/avail.txt ] || timeout -k 10 120 rocprofv3 -L > gpurun_out/avail.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -x -q ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json | head -c 1500; echo
if [ $rc -ne 0 ]; then tail -5 $OUT/bench.err; exit $rc; fi
# the same bench command under the profiler (its JSON line lands in trace.log: its hipEvent
# main_kernel_ms and rocprof's average for the main kernel describe the same launches)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $OUT/trace.log 2>&1
rc=$?; echo "rocprof trace rc=$rc"
if [ $rc -ne 0 ]; then tail -20 $OUT/trace.log; exit $rc; fi
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/trace -name "*kernel_trace.csv" -exec cp {} $OUT/kernel_trace.csv \;
head -20 $OUT/kernel_stats.csv
# the int8 main kernel over bench.py's timed window (its default warm-up calls skipped)
python3 tools/trace_window.py $OUT/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64" 30 50 | tee $OUT/trace_window.txt
i=0
for ctr in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-siblings > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/pmc$i.log; exit $rc; fi
done
exit 0
