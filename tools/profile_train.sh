#!/bin/bash
# Training-step measurement: bench --train (HIP graph and eager, plain and deterministic) + a
# rocprofv3 kernel-trace of the deterministic graph step.  Output: gpurun_out/train_$TAG/
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02}
OUT=$R/gpurun_out/train_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
: > $OUT/train.jsonl
for a in "" "--no-graph" "--deterministic" "--deterministic --no-graph"; do
  timeout -k 10 300 python3 $R/bench.py --train --steps 20 --warmup 3 $a > $OUT/run.log 2> $OUT/run.err || exit $?
  tail -1 $OUT/run.log >> $OUT/train.jsonl
done
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o train -- \
  python3 $R/bench.py --train --deterministic --steps 7 --warmup 1 > $OUT/train_traced.log 2>&1 || exit $?
echo train collected
