#!/bin/bash
# A/B of whole libqmha.so builds on one box: bench.py with the given arguments against the
# default build and each quantizedmha_amd/alt_lib/<name> (tools/alt_build.sh), interleaved twice.
# usage: bash tools/ab_bench.sh <tag> "<alt names>" "<bench.py args>"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=${1:-ab}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for lib in default $2; do
    if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 200 python bench.py --no-siblings --no-cpu-baseline --no-solve-calls $3 > $OUT/${lib}_$rep.json 2>$OUT/${lib}_$rep.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $lib rc=$rc"; tail -3 $OUT/${lib}_$rep.err; exit $rc; }
    python - "$lib" $OUT/${lib}_$rep.json <<'PY'
import json,sys
j=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rc=j.get("reference_config") or {}
print(f"  {sys.argv[1]:12s} step {j['ms_per_step']:.4f} main {j['roofline']['main_kernel_ms']:.4f} pre {j['roofline']['prepass_ms']:.4f}"
      + (f" | refcfg main {rc['main_kernel_ms']:.4f}" if rc else ""))
PY
  done
done
