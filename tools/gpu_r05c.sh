#!/bin/bash
# Round 5: PSMNet-AA near-tie fixture flips per level (default vs exact-f32 engine), then the
# full GPU suite (without -x), smoke and one bench line of the in-tree library.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/diag_raw_flips.py > gpurun_out/raw_flips.txt 2>&1 || { tail -5 gpurun_out/raw_flips.txt; exit 3; }
AANET_EXACT_F32=1 timeout -k 10 200 python tools/diag_raw_flips.py >> gpurun_out/raw_flips.txt 2>&1 || { tail -5 gpurun_out/raw_flips.txt; exit 3; }
cat gpurun_out/raw_flips.txt | grep model_
bash tools/gpu_full.sh
