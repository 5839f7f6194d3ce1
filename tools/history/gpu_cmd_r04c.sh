#!/bin/bash
# r04c: under-filled-grid A/B (one C4 sequence per call) of the d = 64 int8 main kernel's register
# budget / fences / workgroup size, then the HEAD bench under rocprofv3 --kernel-trace --stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r04c; mkdir -p $O
for rep in 1 2 3; do
  for lib in default lb2 lb2nf nf w8lb2; do
    if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 120 python tools/probe_calls.py --reps 10 --bursts batched,async1 > $O/probe_${lib}_$rep.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "$lib rc=$rc"; tail -5 $O/probe_${lib}_$rep.log; exit $rc; }
    echo "$lib rep $rep: $(tail -1 $O/probe_${lib}_$rep.log)"
  done
done | tee $O/ab_summary.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
head -c 1500 $O/bench.json; echo
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -5 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/prof
ls -la $O | head -40
