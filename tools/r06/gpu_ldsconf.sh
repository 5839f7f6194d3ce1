#!/bin/bash
# r06: one PMC pass (LDS bank conflicts) per variant / head size, to find kernels whose LDS reads conflict.
# usage: bash tools/r06/gpu_ldsconf.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06lds}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for run in "fa_tc_int8_b 1 32 8192 32" "fa_tc_int8_b 16 8 4096 128" "fa_tc_int8_pt 1 32 8192 32" "fa_tc_int8_pt 16 8 4096 128" \
           "fa_tc_v1a 1 32 8192 32" "fa_tc_v1a 16 8 4096 128" "fa_tc_v1a 16 16 4096 64" "fa_tc_int8_pt 16 16 4096 64"; do
  set -- $run; n=$1_d$5_B$2
  timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS -d $OUT/$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-siblings --no-refconfig --no-solve-calls --variant $1 --B $2 --H $3 --N $4 --d $5 > $OUT/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$n.log; exit $rc; fi
  python3 tools/pmc_summary.py $OUT/$n --kernel qmha > $OUT/$n.summary.txt 2>&1
  python3 - $OUT/$n.summary.txt <<'PY'
import re, sys
name = None
for line in open(sys.argv[1]):
    if line and not line[0].isspace():
        name = line.strip()[:70]
    m = re.match(r"\s+(SQ_LDS_BANK_CONFLICT|SQ_LDS_IDX_ACTIVE)\s+(\S+)", line)
    if m and name and "kernel" in name:
        print("   ", name, m.group(1), m.group(2))
PY
done
exit 0
