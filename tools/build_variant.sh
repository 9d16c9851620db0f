#!/bin/bash
# Build the working tree's library with extra compile flags as aanet_amd/libaanet_mi355x_<tag>.so
# (a scratch copy of csrc, so the product build/ is untouched), for same-call A/B runs
# (tools/ab_libs.sh).  Usage: [ONLY=dcn_tile.hip] build_variant.sh <tag> "<extra hipcc flags>"
set -e
TAG=$1; EXTRA=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/aanet_amd" "$T/include"
cp -r "$R/aanet_amd/csrc" "$T/aanet_amd/"; cp "$R/include/"*.h "$T/include/"
# ONLY=<src.hip>: reuse the product objects and recompile just that source with the extra flags
if [ -n "$ONLY" ]; then touch "$T/aanet_amd/csrc/$ONLY"; else rm -rf "$T/aanet_amd/csrc/build"; fi
make -s -C "$T/aanet_amd/csrc" -j8 LIB="$R/aanet_amd/libaanet_mi355x_$TAG.so" \
  HIPFLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wall -Wno-unused-function -Xclang -target-feature -Xclang -packed-fp32-ops $EXTRA"
rm -rf "$T"
echo "$R/aanet_amd/libaanet_mi355x_$TAG.so"
