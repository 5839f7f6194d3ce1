#!/bin/bash
# r06: instruction-class hide table (tools/ubench/mfma_fill2.hip) + one bench line with the sysfs sampler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=${1:-r06u}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 tools/ubench/mfma_fill2 > $OUT/ubench_mfma_fill2.txt 2>&1
rc=$?; echo "ubench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/ubench_mfma_fill2.txt; exit $rc; }
head -30 $OUT/ubench_mfma_fill2.txt
timeout -k 10 600 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
python3 -c "import json; j=json.load(open('$OUT/bench.json')); print({k: j.get(k) for k in ('value','ms_per_step','clock_ghz','cycles_per_tile','power_cap_w','sysfs_during_timed_calls')}, j['roofline']['main_kernel_ms'])"
exit 0
