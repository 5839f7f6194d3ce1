#!/bin/bash
# HBM traffic PMC passes (FETCH_SIZE, WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM
# section) for one bench variant; writes gpurun_out/<tag>/pmc_<variant>.json -- copy it to
# profiles/<round>/ (where bench.py reads roofline.traffic from).
# usage: bash tools/pmc_traffic.sh <tag> <round> <variant> B H N d
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; ROUND=$2; VAR=$3; B=$4; H=$5; N=$6; D=$7
OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-siblings --no-refconfig --variant $VAR --B $B --H $H --N $N --d $D > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/pmc$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT --kernel qmha --json-out $OUT/pmc_$VAR.json --shape $B $H $N $D | tee $OUT/summary.txt
