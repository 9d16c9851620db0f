#!/bin/bash
# HIP bilinear resize forward: the resize / training GPU tests, then the training step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine_conv.py tests/test_gpu_train.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05n_pytest.txt 2>&1 || { tail -30 gpurun_out/r05n_pytest.txt; exit 11; }
tail -2 gpurun_out/r05n_pytest.txt
timeout -k 10 300 python bench.py --train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r05n_train.json 2>gpurun_out/r05n_train.err || exit 13
tail -1 gpurun_out/r05n_train.json | cut -c1-330
