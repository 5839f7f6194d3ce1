#!/bin/bash
# d = 32 main-kernel time vs batch (rounds of workgroups): per-tensor and per-block
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/b32
for v in fa_tc_int8_pt fa_tc_int8_b; do for B in 1 2 4 8; do
  timeout -k 10 120 python bench.py --variant $v --B $B --H 32 --N 8192 --d 32 --steps 20 --warmup 20 --no-siblings --no-cpu-baseline --no-solve-calls --no-refconfig > gpurun_out/b32/${v}_B$B.json 2>gpurun_out/b32/${v}_B$B.err || exit $?
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline']; print(sys.argv[2], sys.argv[3], 'main', r['main_kernel_ms'], 'per B', round(r['main_kernel_ms']/int(sys.argv[3]),4))" gpurun_out/b32/${v}_B$B.json $v $B
done; done
bash tools/ab_env.sh b32/ab "--variant fa_tc_int8_pt --B 1 --H 32 --N 8192 --d 32 --steps 20 --warmup 20 --no-refconfig" w4=default w8=pt32w8
