#!/bin/bash
# r05p: blocking solve() via a stream-ordered host-flag write spun on, against hipStreamSynchronize
# (QMHA_SOLVE_SYNC=1) -- the solve() tests, then same-box alternating bursts of 16 one-sequence solve() calls
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c_abi_solve or driver_binary or jax_ext or all_ones" > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
for r in 1 2 3; do
  for m in 0 1; do
    QMHA_SOLVE_SYNC=$m timeout -k 10 150 python tools/probe_calls.py --reps 10 --bursts solve,async1 > $O/probe_s${m}_r$r.txt 2>&1 || { tail -5 $O/probe_s${m}_r$r.txt; exit 1; }
    echo "sync=$m r$r: $(tail -1 $O/probe_s${m}_r$r.txt)"
  done
done
for v in fa_tc_v1a fa; do
  for m in 0 1; do
    QMHA_SOLVE_SYNC=$m timeout -k 10 150 python tools/probe_calls.py --variant $v --reps 10 --bursts solve > $O/probe_${v}_s$m.txt 2>&1 || exit 1
    echo "$v sync=$m: $(tail -1 $O/probe_${v}_s$m.txt)"
  done
done
