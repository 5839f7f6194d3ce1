#!/bin/bash
# r05i: HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the fused int8 and fp16 calls at C4 / C3:
# the one-launch forms move only the algorithmic bytes (no K/V intermediates round trip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/r05i; mkdir -p $O
for v in fa_tc_int8_b fa_tc_v1a; do
  i=0
  for ctr in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    QMHA_FUSED=1 QMHA_F16_FUSED=1 timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/$v/pmc$i -o run --output-format csv -- python3 tools/probe_calls.py --variant $v --reps 3 --bursts batched > $O/${v}_pmc$i.log 2>&1 || { tail -20 $O/${v}_pmc$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py $O/$v --kernel qmha --json-out $O/pmc_fused_$v.json --shape 16 16 4096 64 > $O/summary_$v.txt 2>&1
  grep -E "^[a-zA-Z_]|hbm_" $O/summary_$v.txt
done
