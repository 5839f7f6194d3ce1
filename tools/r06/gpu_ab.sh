#!/bin/bash
# r06 same-box alternating A/B: alt_lib/$BASE vs the current build, C4 and the reference shape.
# usage: bash tools/r06/gpu_ab.sh <tag> <base-alt-lib-name> <variants> [extra shapes...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
TAG=$1; BASE=$2; VARS=$3; shift 3; OUT=gpurun_out/$TAG; mkdir -p $OUT
LIBS=base=quantizedmha_amd/alt_lib/$BASE/libqmha.so,new=quantizedmha_amd/lib/libqmha.so
for shape in 16,4096,16,64 "$@"; do
  timeout -k 10 300 python tools/r06/ab_inproc.py --libs $LIBS --variants $VARS --shape $shape --rounds 8 > $OUT/ab_$shape.txt 2>&1
  rc=$?; echo "ab $shape rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/ab_$shape.txt; exit $rc; }
  python3 - $OUT/ab_$shape.txt <<'PY'
import json, sys
j = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for v, r in j.items():
    print(v, r["shape"], "bit-identical:", r["bit_identical_to_first"],
          {n: (x["main_ms_mean"], x["call_ms_mean"], x["main_vs_first"]) for n, x in r["libs"].items()})
PY
done
exit 0
