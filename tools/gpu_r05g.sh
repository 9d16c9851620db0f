#!/bin/bash
# Round 5: direct few-channel convs (small_conv.hip) -- conv / model / module tests, the full-model
# stage table after the change; then the concat / difference band-height A/B (8 in-tree, 16, 24).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/fm
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv.py \
  tests/test_gpu_models.py tests/test_gpu_modules.py tests/test_gpu_train.py > gpurun_out/pytest_r05g.log 2>&1
rc=$?; tail -6 gpurun_out/pytest_r05g.log; [ $rc -le 1 ] || exit $rc
for m in aanet aanetplus; do
  timeout -k 10 300 python tools/full_model_stages.py $m --iters 5 > gpurun_out/fm/stages2_$m.txt 2>&1 || { tail -5 gpurun_out/fm/stages2_$m.txt; exit 3; }
  grep -v "^{" gpurun_out/fm/stages2_$m.txt | grep -v "Warning\|warn\|amdgpu.ids\|_cuda_set"
done
for r in 1 2; do
  timeout -k 10 120 python tools/shift_bench.py 20 || exit 4
  for v in 16 24; do AANET_MI355X_LIB=$PWD/abl/libyb$v.so timeout -k 10 120 python tools/shift_bench.py 20 || exit 4; done
done
exit $rc
