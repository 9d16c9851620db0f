#!/bin/bash
# HIP-graph replay of the eval step under the HIP runtime's graph-execution knobs, vs eager:
#   bash tools/ab_graph_env.sh
mkdir -p gpurun_out
one() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 3 --no-cpu-baseline $BARGS 2>/dev/null > gpurun_out/ge.json || { echo "$label failed"; return 0; }
  python -c "import json; d=json.loads(open('gpurun_out/ge.json').read().strip().splitlines()[-1]); print('$label', round(d['ms_per_step'],4), d['config']['schedule'])"
}
for r in 1 2; do
  BARGS="--no-graph" one eager X=1
  BARGS="--graph" one graph_default X=1
  BARGS="--graph" one graph_nopacket DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
  BARGS="--graph" one graph_q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4
  BARGS="--graph" one graph_q3 DEBUG_HIP_FORCE_GRAPH_QUEUES=3
  BARGS="--graph" one graph_q4_nopacket DEBUG_HIP_FORCE_GRAPH_QUEUES=4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
done
