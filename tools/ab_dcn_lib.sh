#!/bin/bash
# Same-call A/B of two library builds on the scale-0 window DCN tail and the whole bench step:
#   bash tools/ab_dcn_lib.sh <lib_a.so> <lib_b.so> [rounds]
A=$1; B=$2; ROUNDS=${3:-2}
for r in $(seq $ROUNDS); do
  for L in $A $B; do
    echo "== $(basename $L) round $r: dcn_tile_bench"
    AANET_MI355X_LIB=$L timeout -k 10 120 python tools/dcn_tile_bench.py 20 0.5 || exit $?
  done
done
for r in $(seq $ROUNDS); do
  for L in $A $B; do
    echo "== $(basename $L) round $r: bench"
    AANET_MI355X_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline || exit $?
  done
done
