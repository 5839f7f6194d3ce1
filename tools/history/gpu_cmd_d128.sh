#!/bin/bash
# per-tensor vs per-block int8 at d = 128 (B16 H8 N4096) and d = 32 (B16 H32 N4096)
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/dsz
for cfg in "--B 16 --H 8 --N 4096 --d 128" "--B 16 --H 32 --N 4096 --d 32"; do for v in fa_tc_int8_pt fa_tc_int8_b; do
  tag=$(echo "$v $cfg" | tr -d ' -')
  timeout -k 10 120 python bench.py --variant $v $cfg --steps 20 --warmup 20 --no-siblings --no-cpu-baseline --no-solve-calls --no-refconfig > gpurun_out/dsz/$tag.json 2>gpurun_out/dsz/$tag.err || exit $?
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline']; print(sys.argv[2], 'main', r['main_kernel_ms'], 'pre', r['prepass_ms'], 'frac', r['frac'])" gpurun_out/dsz/$tag.json "$v $cfg"
done; done
