#!/bin/bash
# A/B an environment switch of the conv engine within ONE GPU call (boxes differ in clocks):
#   bash tools/ab_env.sh VAR "val1 val2 ..." cases [rounds]
VAR=$1; VALS=$2; CASES=$3; ROUNDS=${4:-2}
for r in $(seq $ROUNDS); do
  for v in $VALS; do
    echo "== $VAR=$v round $r"
    env $VAR=$v timeout -k 10 300 python tools/conv_microbench.py 20 $CASES || exit $?
  done
done
