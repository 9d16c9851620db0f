#!/bin/bash
# LDS-DMA barrier fix: kernel determinism beside other work, the full step's concurrent-schedule
# determinism, the affected kernels' tests, then the step A/B against abl/libhead.so.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N=40 timeout -k 10 300 python tools/race_probe.py 2>&1 | grep -v amdgpu.ids || exit 3
PROBE_DEFAULT_ONLY=1 timeout -k 10 200 python tools/nondet_probe.py 2>&1 | tail -1 || exit 4
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_g3.py tests/test_gpu_conv_s2.py tests/test_gpu_production.py 2>&1 | tail -1 || exit 5
bash tools/gpu_r05u.sh
