#!/bin/bash
# Concat band kernel A/B, planes d and d+D/2 alternating (in-tree) vs d order (abl/libhead.so):
# the shift-volume tests, then the C5 concat live time from the bench kernel loops, 3 rounds.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py 2>&1 | tail -1 || exit 3
for r in 1 2 3; do
for L in aanet_amd/libaanet_mi355x.so abl/libhead.so; do
  AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --kernel-iters 30 2>/dev/null > gpurun_out/ab_lib.json || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1]); k=d['kernels']['concat_volume_c5']
print('$L concat_c5 %.1f us frac %.3f' % (k['ms']*1e3, k['frac']))"
done
done
