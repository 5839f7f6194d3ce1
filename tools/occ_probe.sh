cd "${GRAFT_REPO_ROOT}"
for pad in 0 20000 50000 0; do
  QMHA_LIB_PATH=$PWD/quantizedmha_amd/alt_lib/abl/libqmha.so QMHA_INT8_LDS_PAD=$pad timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-siblings --no-cpu-baseline > gpurun_out/occ_$pad.json 2>gpurun_out/occ_$pad.err || exit 1
  python3 -c "import json,sys; j=json.load(open('gpurun_out/occ_$pad.json')); print('pad $pad main', j['roofline']['main_kernel_ms'])"
done
