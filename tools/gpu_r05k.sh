#!/bin/bash
# DCN backward A/B: the window-form DCN GPU tests, then the C4 sweep timings (no profiler).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mdcn.py -x -q --timeout 300 --timeout-method thread -k "backward" > gpurun_out/r05k_pytest.txt 2>&1 || { tail -30 gpurun_out/r05k_pytest.txt; exit 11; }
tail -2 gpurun_out/r05k_pytest.txt
timeout -k 10 300 python3 bench.py --dcn-sweep --kernel-iters 10 > gpurun_out/r05k_sweep.jsonl 2>gpurun_out/r05k_sweep.err || exit 12
cat gpurun_out/r05k_sweep.jsonl
