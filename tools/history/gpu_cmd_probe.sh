cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 240 python3 tools/probe_calls.py --reps 5 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -3 $O/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 tools/probe_calls.py --reps 5 > $O/probe_prof.log 2>&1 || { tail -20 $O/probe_prof.log; exit 1; }
find $O/trace -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/trace
ls -la $O
