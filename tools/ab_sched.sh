#!/bin/bash
# Interleaved A/B of the conv-engine schedule variants (same process order alternated).
set -u
for r in 1 2; do
  for v in 0 1; do
    echo "== AANET_SCHED=$v round $r"
    AANET_SCHED=$v timeout -k 10 300 python tools/conv_microbench.py 20 || exit $?
  done
done
