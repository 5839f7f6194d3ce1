#!/bin/bash
# r04h: HEAD bench (default arguments, every side measurement) and the same bench under
# rocprofv3 --kernel-trace --stats; timed-window average of the headline main kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/trace
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi65E" 30 50 | tee $O/trace_window.txt
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi1048641E" 30 50 | tee -a $O/trace_window.txt
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_f16_v2_kernelILi64" 30 50 | tee -a $O/trace_window.txt
