#!/bin/bash
# Stride-2 kernel check: its GPU tests, the microbenchmark (rolled vs straight-line form), the
# production parity tests, then one bench line.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_s2.py tests/test_gpu_production.py > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2_tests.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0 1; do AANET_S2_ROWS=$f timeout -k 10 120 python tools/s2_bench.py | sed "s/^/rows=$f /" || exit 1; done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print('bench', round(d['ms_per_step'],4), 'ms', round(d['value'],1), 'pairs/s', d['config']['schedule'], 'epe', d['epe_vs_ref'], d['max_abs_disp_err_vs_ref'])"
