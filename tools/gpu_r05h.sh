#!/bin/bash
# Round 5: hoisted CSA epilogue geometry (engine + DCN tail) -- tests, then the bench-step A/B
# against abl/libold.so (the previous commit's library)
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py \
  tests/test_gpu_production.py tests/test_gpu_dcn_tile.py tests/test_gpu_post.py tests/test_gpu_split.py \
  tests/test_gpu_engine_conv.py > gpurun_out/pytest_r05h.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r05h.log; [ $rc -le 1 ] || exit $rc
bash tools/ab_step.sh || exit 5
exit $rc
