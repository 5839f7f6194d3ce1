#!/bin/bash
# d = 64 main-kernel time vs batch: fixed per-launch overhead of the int8 kernels
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/b64
for v in fa_tc_int8_b fa_tc_int8_pt; do for B in 2 4 8 16 32 64; do
  timeout -k 10 120 python bench.py --variant $v --B $B --H 16 --N 4096 --d 64 --steps 20 --warmup 20 --no-siblings --no-cpu-baseline --no-solve-calls --no-refconfig > gpurun_out/b64/${v}_B$B.json 2>gpurun_out/b64/${v}_B$B.err || exit $?
  python -c "import json,sys; j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=j['roofline']; print(sys.argv[2], sys.argv[3], 'main', r['main_kernel_ms'], 'per B', round(r['main_kernel_ms']/int(sys.argv[3]),5))" gpurun_out/b64/${v}_B$B.json $v $B
done; done
export QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/tl/libqmha.so
for args in "fa_tc_int8_b 1 32 8192 32" "fa_tc_int8_pt 1 32 8192 32" "fa_tc_int8_b 16 16 4096 64" "fa_tc_int8_pt 16 16 4096 64" "fa_tc_int8_b 4 32 8192 32"; do
  timeout -k 10 120 python tools/timeline.py $args > gpurun_out/b64/tl_$(echo $args | tr ' ' '_').txt 2>&1 || { cat gpurun_out/b64/tl_$(echo $args | tr ' ' '_').txt | tail -5; exit 1; }
  cat gpurun_out/b64/tl_$(echo $args | tr ' ' '_').txt
done
