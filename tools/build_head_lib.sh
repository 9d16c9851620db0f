#!/bin/bash
# Build the library of a git revision (default HEAD) as aanet_amd/libaanet_mi355x_<tag>.so, for
# same-call A/B runs against the working tree (tools/ab_lib.sh).  Usage: build_head_lib.sh [rev] [tag]
set -e
REV=${1:-HEAD}; TAG=${2:-head}
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
git -C "$R" archive "$REV" aanet_amd/csrc include | tar -x -C "$T"
make -s -C "$T/aanet_amd/csrc" -j8 LIB="$R/aanet_amd/libaanet_mi355x_$TAG.so"
rm -rf "$T"
echo "$R/aanet_amd/libaanet_mi355x_$TAG.so"
