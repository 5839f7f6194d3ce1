#!/bin/bash
# r05f: HEAD evidence -- full GPU suite + smoke, HBM PMC passes (int8 per-block, per-tensor, fp16 at C4), SQ
# passes (both int8 kernels), the bench, the bench under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
T=${1:-r05f}; O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_cmd_tests.sh $T || exit $?
for v in fa_tc_int8_b fa_tc_int8_pt fa_tc_v1a; do
  bash tools/pmc_traffic.sh ${T}_$v r05 $v 16 16 4096 64 > $O/pmc_traffic_$v.txt 2>&1 || { tail -20 $O/pmc_traffic_$v.txt; exit 1; }
done
for v in fa_tc_int8_b fa_tc_int8_pt; do
  BENCH_ARGS="--no-solve-calls --variant $v" bash tools/pmc_sq.sh ${T}_sq_$v > /dev/null || exit $?
  python3 tools/pmc_summary.py gpurun_out/${T}_sq_$v --kernel qmha --json-out gpurun_out/${T}_sq_$v/pmc_sq_$v.json --shape 16 16 4096 64 > gpurun_out/${T}_sq_$v/summary.txt || exit $?
done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 600 $O/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/trace
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi65E" 30 50 | tee $O/trace_window.txt
ls gpurun_out/${T}_*/*.json
