#!/bin/bash
# Offset-conv kernel check: its GPU tests, the production/DCN parity tests, then the bench step
# with the kernel on and off (AANET_OFFSET_KERNEL).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_g3.py tests/test_gpu_production.py tests/test_gpu_dcn_tile.py > gpurun_out/g3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g3_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1 0; do AANET_OFFSET_KERNEL=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-iters 10 > gpurun_out/bench_g3_$f.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('gpurun_out/bench_g3_$f.log').read().strip().splitlines()[-1]); print('offset_kernel=$f bench', round(d['ms_per_step'],4), d['config']['schedule'], 'epe', d['epe_vs_ref'], d['max_abs_disp_err_vs_ref'])"; done
