#!/bin/bash
# Round 4: pre-split NCHW pointwise conv -- pointwise / post / production tests, then a same-call
# A/B of the bench step and its conv1x1_s0 line (base = pre-split, pwold = -DPW_PRESPLIT=0).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_pointwise.py tests/test_gpu_post.py tests/test_gpu_production.py tests/test_gpu_modules.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04q_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for V in ${VARS:-base pwold}; do
    L=aanet_amd/libaanet_mi355x_$V.so; [ $V = base ] && L=aanet_amd/libaanet_mi355x.so
    AANET_MI355X_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04q_$V.json 2>&1 || exit 8
    python -c "import json; d=json.loads(open('gpurun_out/r04q_$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$V', round(d['ms_per_step'],4), 'ms', 'conv1x1', round(k['conv1x1_s0']['ms']*1e3,1), 'us frac', round(k['conv1x1_s0']['frac'],3), 'epe', d['epe_vs_ref'])"
  done
done
