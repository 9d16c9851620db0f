#!/bin/bash
# Training step: MIOpen plain convs (auto) vs the HIP engine for every plain conv (on).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for e in auto on; do
  timeout -k 10 300 python bench.py --train --engine-convs $e --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05o_train_$e.json 2>gpurun_out/r05o_train_$e.err || exit 13
  tail -1 gpurun_out/r05o_train_$e.json | cut -c1-330
done
