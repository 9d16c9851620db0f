#!/bin/bash
# Round 5: concat / difference band height A/B (AANET_BAND_ROWS 8 in-tree, 16, 24) at C5
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 120 python tools/shift_bench.py 20 || exit 4
  for v in 16 24; do AANET_MI355X_LIB=$PWD/abl/libyb$v.so timeout -k 10 120 python tools/shift_bench.py 20 || exit 4; done
done
