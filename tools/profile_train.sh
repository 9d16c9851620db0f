#!/bin/bash
# Training-step measurement: bench --train (plain and deterministic) + a rocprofv3 kernel-trace of it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r01}
OUT=$R/gpurun_out/train_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --train --steps 10 --warmup 3 > $OUT/train.json 2> $OUT/train.err || exit $?
timeout -k 10 300 python3 $R/bench.py --train --deterministic --steps 10 --warmup 3 > $OUT/train_det.json 2> $OUT/train_det.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o train -- \
  python3 $R/bench.py --train --steps 5 --warmup 2 > $OUT/train_traced.log 2>&1 || exit $?
cat $OUT/train.json $OUT/train_det.json
