#!/bin/bash
# Round 4: the offset conv's 32x32x16 wide form -- tests, alone (g3_bench), and same-call A/B of
# the bench step against the 16x16x32 form (-DG3_WIDE=0 build).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_g3.py tests/test_gpu_production.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04k_tests.log 2>&1
rc=$?; tail -4 gpurun_out/r04k_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 100 python tools/g3_bench.py || exit 6
  AANET_MI355X_LIB=aanet_amd/libaanet_mi355x_g3old.so timeout -k 10 100 python tools/g3_bench.py || exit 6
done
VARS="base g3old" bash tools/gpu_r04i.sh 2>&1 | grep -E "^(base|g3old) " 
