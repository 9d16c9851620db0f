#!/bin/bash
# DCN tail epilogue on buffer resources: the DCN tile / production / model tests, then a same-call
# A/B of the bench step against abl/libhead.so (live per-kernel times).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
true
true
for r in 1 2 3; do
for L in aanet_amd/libaanet_mi355x.so abl/libhead.so; do
  AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null > gpurun_out/ab_lib.json || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$L', round(d['ms_per_step'],4), 'ms/step;', '; '.join('%s %.1f us %.3f' % (n, k[n]['ms']*1e3, k[n]['frac']) for n in ('mdcn_pw_s0','conv3x3_pw_s0','offset_conv_s0') if n in k))"
done
done
