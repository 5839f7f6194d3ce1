#!/bin/bash
# r06: one default bench line on the current tree (box spread at HEAD): clock probe, sysfs, isa_sha16.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r06bench}; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/bench.err; exit $rc; }
python3 -c "import json; j=json.load(open('$O/bench.json')); s=j['siblings']; print(j['device']['pci'], j['ms_per_step'], j['roofline']['main_kernel_ms'], j['clock_ghz'], j['cycles_per_tile'], s['fa_tc_v1a']['main_kernel_ms'], s['fa_tc_int8_pt']['main_kernel_ms'], s['fa_tc_int8_pt']['ms_per_step'])"
