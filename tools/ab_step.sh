#!/bin/bash
# Same-call A/B of two library builds on the bench step: abl/libold.so (AANET_MI355X_LIB) vs the
# in-tree build, alternating, plus an optional dcn_tile microbench.  Usage: bash tools/ab_step.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export AANET_MI355X_LIB=$PWD/abl/libold.so; else unset AANET_MI355X_LIB; fi
    timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit 4
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$v', round(d['ms_per_step'],4), 'dcn', round(k['mdcn_pw_s0']['ms']*1e3,1), 'heads', round(k['s2_heads_s0']['ms']*1e3,1), 'g3', round(k['offset_conv_s0']['ms']*1e3,1), 'tail', round(k['conv3x3_pw_s0']['ms']*1e3,1))"
  done
done
unset AANET_MI355X_LIB
