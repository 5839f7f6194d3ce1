#!/bin/bash
# Runtime occupancy of the int8/f16 main kernels in a built object (runs on the GPU box).
# usage: bash tools/occ.sh <obj.o> <block> <kernel-substring>...
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OBJ=$1; BLOCK=$2; shift 2
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin $OBJ
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
NAMES=""
for p in "$@"; do NAMES="$NAMES $(/opt/rocm/lib/llvm/bin/llvm-readelf --syms $T/k.co | awk "{print \$8}" | grep -v "\.kd$" | grep -- "$p" | head -1)"; done
tools/ubench/occupancy $T/k.co $BLOCK $NAMES
