#!/bin/bash
# Same-call A/B of two builds of the library: bash tools/ab_lib.sh <lib_a.so> <lib_b.so> cases [rounds]
A=$1; B=$2; CASES=$3; ROUNDS=${4:-2}
for r in $(seq $ROUNDS); do
  for L in $A $B; do
    echo "== $(basename $L) round $r"
    AANET_MI355X_LIB=$L timeout -k 10 300 python tools/conv_microbench.py 20 $CASES || exit $?
  done
done
