#!/bin/bash
# r04u: HEAD with the fused per-block int8 kernel (FL_FUSED): its bit-identity test,
# the full GPU suite + smoke, a same-box alternating A/B of the calling patterns (QMHA_FUSED 0 / 1),
# the HEAD bench, the bench under rocprofv3 --kernel-trace --stats, HBM PMC passes of the fused kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_zfused.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_fused.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests_fused.log | tail -1; [ $rc -ne 0 ] && { tail -40 $O/tests_fused.log; exit $rc; }
bash tools/gpu_cmd_tests.sh r04u || exit $?
for r in 1 2; do
  for m in 0 1; do
    QMHA_FUSED=$m timeout -k 10 150 python tools/probe_calls.py --reps 10 > $O/probe_m${m}_r$r.txt 2>&1 || { tail -5 $O/probe_m${m}_r$r.txt; exit 1; }
    echo "fused=$m round $r: $(tail -1 $O/probe_m${m}_r$r.txt)"
  done
done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 900 $O/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-solve-calls > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/trace
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi2097217E" 30 50 | tee $O/trace_window.txt
python3 tools/trace_window.py $O/kernel_trace.csv "qmha_fa_int8_pipe_kernelILi64ELi4ELi1048641E" 30 50 | tee -a $O/trace_window.txt
bash tools/pmc_traffic.sh r04u_pmc r04 fa_tc_int8_b 16 16 4096 64 || exit $?
