#!/bin/bash
# Conv weight-gradient workgroup target A/B: the training step with the in-tree library (2048)
# and abl/libw{512,768,1024}.so (built with -DAANET_WGRAD_WGS=...), 2 rounds.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for r in 1 2; do
for L in aanet_amd/libaanet_mi355x.so abl/libw512.so abl/libw768.so abl/libw1024.so; do
  AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null > gpurun_out/ab_w.json || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_w.json').read().strip().splitlines()[-1])
print('$L train %.3f ms' % d['ms_per_step'])"
done
done
