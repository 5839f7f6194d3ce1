#!/bin/bash
# Build an A/B variant of libqmha.so with extra flags into quantizedmha_amd/alt_lib/<name>/
# (own object directory build/obj_<name>; the production build is left untouched)
# usage: bash tools/alt_build.sh <name> "<extra hipcc flags>"
set -e
cd "$(dirname "$0")/.."
rm -rf "build/obj_$1"  # flags are not tracked by the incremental build
QMHA_ALT="$1" QMHA_EXTRA_FLAGS="$2" python tools/build.py
echo "alt/$1 built with: $2"
