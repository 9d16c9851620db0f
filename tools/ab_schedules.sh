#!/bin/bash
# Step time of the eval schedules (HIP graph vs eager; side streams per coarse scale / one shared /
# none): bash tools/ab_schedules.sh [rounds]
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BARGS 2>/dev/null > gpurun_out/ab_sched.json || return 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_sched.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), 'ms/step', round(d['value'],1), 'pairs/s graph', d['config'].get('hip_graph'))"
}
for r in $(seq ${1:-1}); do
  BARGS="" run graph_2side AANET_SIDE_STREAMS=0 || exit 1
  BARGS="--no-graph" run eager_2side AANET_SIDE_STREAMS=0 || exit 1
  BARGS="" run graph_1side AANET_SIDE_STREAMS=1 || exit 1
  BARGS="--no-graph" run eager_1side AANET_SIDE_STREAMS=1 || exit 1
  BARGS="" run graph_serial AANET_CONCURRENT_SCALES=0 || exit 1
done
