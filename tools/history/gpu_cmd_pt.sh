#!/bin/bash
# per-tensor int8 mode (fa_tc_int8_pt): parity subset, then a short bench against fa_tc_int8_b
cd $GRAFT_REPO_ROOT; export PYTHONUNBUFFERED=1; mkdir -p gpurun_out/pt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -k "int8_pt" > gpurun_out/pt/tests.log 2>&1; rc=$?
echo "pt tests rc=$rc: $(tail -1 gpurun_out/pt/tests.log)"; grep -E "FAILED|Error" gpurun_out/pt/tests.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for v in fa_tc_int8_pt fa_tc_int8_b; do
  timeout -k 10 200 python bench.py --variant $v --steps 20 --warmup 10 --no-siblings --no-cpu-baseline --no-refconfig > gpurun_out/pt/bench_$v.json 2> gpurun_out/pt/bench_$v.err; rc2=$?
  [ $rc2 -ne 0 ] && { tail -5 gpurun_out/pt/bench_$v.err; exit $rc2; }
  python3 -c "import json; j=json.loads(open('gpurun_out/pt/bench_$v.json').read().strip().splitlines()[-1]); r=j['roofline']; print('$v', j['ms_per_step'], 'main', r['main_kernel_ms'], 'pre', r['prepass_ms'], 'frac', r['frac'])"
done
exit $rc
