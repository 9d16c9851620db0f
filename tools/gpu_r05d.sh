#!/bin/bash
# Round 5: DCN tail A/B -- abl/libold.so (the committed library) vs abl/libunroll.so (chunk loop
# fully unrolled, AANET_DCN_UNROLL): the tail alone (tools/dcn_tile_bench.py) and the bench step.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
ROUNDS=3 bash tools/ab_libs.sh $PWD/abl/libold.so $PWD/abl/libunroll.so || exit 5
