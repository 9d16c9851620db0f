#!/bin/bash
# rocprofv3 kernel trace of the training step only (bench --train).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT_NAME:-train_trace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o train -- \
  python3 $R/bench.py --train --steps 5 --warmup 2 ${EXTRA:-} > $OUT/train_traced.log 2>&1 || exit $?
tail -1 $OUT/train_traced.log
