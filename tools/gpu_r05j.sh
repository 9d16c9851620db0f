#!/bin/bash
# Round 5: chunked deterministic DCN backward (int64 weight-gradient accumulator): the DCN GPU
# tests, the training tests, then the C4 sweep and the deterministic training step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mdcn.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05j_pytest.txt 2>&1 || { tail -30 gpurun_out/r05j_pytest.txt; exit 11; }
tail -3 gpurun_out/r05j_pytest.txt
cd $R && bash tools/c4_sweep.sh || exit 12
timeout -k 10 300 python bench.py --train --deterministic --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05j_train_det.json 2>gpurun_out/r05j_train_det.err || exit 14
tail -1 gpurun_out/r05j_train_det.json
echo r05j done
