#!/bin/bash
# Timing attribution of the window DCN tail: AANET_DCN_DBG bits (1 no MFMA, 2 no window reads,
# 4 no fallback, 8 no per-tap barrier, 16 no epilogue traffic, 32 no window loads, 64 no weight
# DMA) at bench-like offsets.  Results are wrong with any bit set: timing only.
for d in ${DBGS:-0 1 7 16 32 64 23 39 71 119 127}; do
  echo "== AANET_DCN_DBG=$d"
  AANET_DCN_DBG=$d timeout -k 5 60 python tools/dcn_tile_bench.py 20 ${SCALES:-0.5} || exit $?
done
