#!/bin/bash
# Kernel-trace profile of bench.py (eager launches so every kernel is attributed).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-prof_step}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $R/bench.py ${BENCH_ARGS:---steps 5 --warmup 2 --no-graph --no-cpu-baseline} > $OUT/bench.log 2>&1
rc=$?
tail -3 $OUT/bench.log
find $OUT -name "*kernel_stats.csv" | head -3
exit $rc
