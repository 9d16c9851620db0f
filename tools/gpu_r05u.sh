#!/bin/bash
# Same-call A/B of the bench step: in-tree library vs abl/libhead.so (3 rounds).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for r in 1 2 3; do
for L in aanet_amd/libaanet_mi355x.so abl/libhead.so; do
  AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline --kernel-iters 5 2>/dev/null > gpurun_out/ab_lib.json || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1])
print('$L', round(d['ms_per_step'],4), 'ms/step', d['config']['schedule'])"
done
done
