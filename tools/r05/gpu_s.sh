#!/bin/bash
# r05v: box-to-box spread -- the box's power cap and clocks (rocm-smi) beside one default bench run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/${1:-r05v}; mkdir -p $O
timeout -k 10 60 rocm-smi --showmaxpower --showpower --showclocks --showproductname > $O/smi_before.txt 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 60 rocm-smi --showmaxpower --showpower --showclocks > $O/smi_after.txt 2>&1
grep -iE "max graphics package power|sclk|socclk|mclk|current socket|Card Series|Card SKU" $O/smi_before.txt | head -12
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().splitlines()[-1]); r=d['roofline']
print('call', d['ms_per_step'], 'main', r['main_kernel_ms'], 'prepass', r['prepass_ms'], 'fp16 main', d['siblings']['fa_tc_v1a']['main_kernel_ms'])"
