#!/bin/bash
# Build the library of git revision REV into abl/lib<NAME>.so for same-call A/B runs:
#   bash tools/build_ab.sh REV NAME
set -eu
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/abtree.XXXX)
mkdir -p $T/aanet_amd/csrc $T/include $R/abl
git -C $R archive $REV aanet_amd/csrc include | tar -x -C $T
make -s -C $T/aanet_amd/csrc -j8 LIB=$R/abl/lib$NAME.so >/dev/null
rm -rf $T
echo "abl/lib$NAME.so from $(git -C $R rev-parse --short $REV)"
