#!/bin/bash
# round-4 evidence session: VALU-cost ubench, the default bench line, and the same bench under rocprofv3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r04b}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 120 tools/ubench/valu_cost > $O/ubench_valu_cost.txt 2>&1 || { tail $O/ubench_valu_cost.txt; exit 1; }
tail -8 $O/ubench_valu_cost.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/trace
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi65E" 30 50 | tee $O/trace_window.txt
