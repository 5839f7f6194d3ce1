#!/bin/bash
# Same-box alternating A/B of libqmha.so builds (quantizedmha_amd/alt_lib/<name>/, "default" = the
# production build) on one variant: REPS rounds, each lib once per round, bench.py's hipEvent
# main-kernel / pre-pass times and ms per call.
# usage: bash tools/ab_run.sh <tag> <variant> "<libs>" [reps] [extra bench.py args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONUNBUFFERED=1
TAG=$1; VAR=$2; LIBS=$3; REPS=${4:-3}; EXTRA=${5:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for lib in $LIBS; do
    if [ "$lib" = default ]; then LP=""; else LP=$PWD/quantizedmha_amd/alt_lib/$lib/libqmha.so; fi
    env QMHA_LIB_PATH=$LP timeout -k 10 180 python bench.py --variant $VAR --steps 20 --warmup 20 --no-siblings \
        --no-cpu-baseline --no-solve-calls --no-refconfig $EXTRA > $OUT/${lib}_$rep.json 2> $OUT/${lib}_$rep.err
    rc=$?; if [ $rc -ne 0 ]; then echo "$lib rep $rep rc=$rc"; tail -5 $OUT/${lib}_$rep.err; exit $rc; fi
    python3 - $lib $rep $OUT/${lib}_$rep.json <<'PY'
import json, sys
j = json.load(open(sys.argv[3])); r = j["roofline"]
print(f"{sys.argv[1]:>16s} rep {sys.argv[2]}: call {j['ms_per_step']:.4f} ms  main {r['main_kernel_ms']:.4f}  pre {r['prepass_ms']:.4f}  frac {r['frac']:.4f}")
PY
  done
done | tee $OUT/summary.txt
