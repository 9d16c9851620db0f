#!/bin/bash
# Timing attribution of the window DCN tail: AANET_DCN_DBG bits (1 no MFMA, 2 no window reads,
# 4 no fallback, 8 no per-tap barrier) over offset statistics.
set -e
for d in 0 4 1 2 8 6 7; do
  echo "== AANET_DCN_DBG=$d"
  AANET_DCN_DBG=$d timeout -k 10 120 python tools/dcn_tile_bench.py 20 ${SCALES:-0,0.5,1.0}
done
