#!/bin/bash
# A/B on one box, interleaved twice: bench.py <args> under each arm.  An arm is
#   name=ALTLIB:ENV1=v1,ENV2=v2     (ALTLIB: quantizedmha_amd/alt_lib/<ALTLIB>/libqmha.so, or "default")
# usage: bash tools/ab_env.sh <tag> "<bench.py args>" arm1 arm2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=$1; ARGS=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for arm in "$@"; do
    name=${arm%%=*}; rest=${arm#*=}; lib=${rest%%:*}; envs=${rest#*:}
    [ "$envs" = "$rest" ] && envs=""
    LP=""; [ "$lib" != default ] && LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so
    env QMHA_LIB_PATH=$LP ${envs//,/ } timeout -k 10 240 python bench.py --no-siblings --no-cpu-baseline --no-solve-calls $ARGS > $OUT/${name}_$rep.json 2>$OUT/${name}_$rep.err
    rc=$?; [ $rc -ne 0 ] && { echo "bench $name rc=$rc"; tail -3 $OUT/${name}_$rep.err; exit $rc; }
    python - "$name" $OUT/${name}_$rep.json <<'PY'
import json,sys
j=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rc=j.get("reference_config") or {}
print(f"  {sys.argv[1]:14s} step {j['ms_per_step']:.4f} main {j['roofline']['main_kernel_ms']:.4f} pre {j['roofline']['prepass_ms']:.4f}"
      + (f" | refcfg main {rc['main_kernel_ms']:.4f}" if rc else ""), flush=True)
PY
  done
done
