#!/bin/bash
# A/B of the split heads schedule (AANET_EARLY_CONV1): production parity with it on, then
# alternating bench runs.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
AANET_EARLY_CONV1=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_production.py > gpurun_out/early_tests.log 2>&1
rc=$?; tail -2 gpurun_out/early_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for f in 0 1; do
  AANET_EARLY_CONV1=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-iters 5 > gpurun_out/ab_early_$f.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_early_$f.log').read().strip().splitlines()[-1]); print('early=$f', round(d['ms_per_step'],4), d['config']['schedule'], d['epe_vs_ref'])"
done; done
