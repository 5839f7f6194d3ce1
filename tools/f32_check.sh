#!/bin/bash
# fp32 sibling: GPU parity tests, then the bench siblings line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-f32}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $OUT/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-solve-calls > $OUT/bench.json 2> $OUT/bench.err
rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/bench.err; exit $rc; }
python -c "import json,sys; j=json.load(open(sys.argv[1])); print(json.dumps(j['siblings'])); print(j['ms_per_step'], j['roofline']['main_kernel_ms'])" $OUT/bench.json
