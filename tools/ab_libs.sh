#!/bin/bash
# Same-call A/B of N library builds on the window DCN tail alone and on the bench step:
#   ROUNDS=2 bash tools/ab_libs.sh lib_a.so lib_b.so [lib_c.so ...]
for r in $(seq ${ROUNDS:-2}); do
  for L in "$@"; do
    echo "== $(basename $L) round $r: $(AANET_MI355X_LIB=$L timeout -k 10 120 python tools/dcn_tile_bench.py 20 0.5 2>/dev/null | tail -1)" || exit 1
  done
done
for L in "$@"; do
  AANET_MI355X_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null > gpurun_out/ab_lib.json || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1]); print('$(basename $L) bench', round(d['ms_per_step'],4), 'ms/step; mdcn_pw_s0', round(d['kernels']['mdcn_pw_s0']['ms']*1e3,1), 'us frac', round(d['kernels']['mdcn_pw_s0']['frac'],4))"
done
