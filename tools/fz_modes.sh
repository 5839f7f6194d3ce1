cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/fz
for f in 0 1 2; do
  timeout -k 10 180 python bench.py --int8-fused $f --steps 10 --warmup 10 --no-siblings --no-cpu-baseline --no-refconfig --no-solve-calls > gpurun_out/fz/b$f.json 2> gpurun_out/fz/b$f.err || exit 1
  python -c "import json,sys; j=json.load(open(sys.argv[1])); r=j['roofline']; print('mode', sys.argv[2], j['ms_per_step'], 'main', r['main_kernel_ms'], 'pre', r['prepass_ms'])" gpurun_out/fz/b$f.json $f
done
