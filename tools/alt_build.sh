#!/bin/bash
# Build an A/B variant of libqmha.so with extra flags into quantizedmha_amd/alt_lib/<name>/
# usage: bash tools/alt_build.sh <name> "<extra hipcc flags>"   (then rebuild the default)
set -e
cd "$(dirname "$0")/.."
QMHA_EXTRA_FLAGS="$2" python tools/build.py --clean > /dev/null
mkdir -p quantizedmha_amd/alt_lib/$1
cp quantizedmha_amd/lib/libqmha.so quantizedmha_amd/alt_lib/$1/
echo "alt/$1 built with: $2"
