#!/bin/bash
# Round 5 profiles: bench kernel stats + PMC passes (profiles/r05_*), the SURVEY C4 DCN sweep, and
# the training step (float and deterministic).  Each step has its own time limit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=r05 bash tools/collect_profiles.sh || exit 11
cd $R && bash tools/c4_sweep.sh || exit 12
cd $R && timeout -k 10 300 python bench.py --train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05_train.json 2>gpurun_out/r05_train.err || exit 13
timeout -k 10 300 python bench.py --train --deterministic --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05_train_det.json 2>gpurun_out/r05_train_det.err || exit 14
tail -1 gpurun_out/r05_train.json; tail -1 gpurun_out/r05_train_det.json
echo r05i done
