#!/bin/bash
# Same-call A/B of an environment switch on the bench step: bash tools/ab_env_bench.sh VAR "a b" [rounds]
VAR=$1; VALS=$2; ROUNDS=${3:-2}
for r in $(seq $ROUNDS); do
  for v in $VALS; do
    echo "== $VAR=$v round $r"
    env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.json 2>/dev/null || exit $?
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'ms/step', round(d['value'],1), 'pairs/s', 'epe', d.get('epe_vs_ref'), 'max', d.get('max_abs_disp_err_vs_ref'))"
  done
done
