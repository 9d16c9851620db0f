#!/bin/bash
# Inference step kernel breakdown: rocprofv3 kernel trace of the bench step (HIP graph replays).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/step_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/step_prof -o st -- \
  python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --kernel-iters 1 > $R/gpurun_out/step_prof/log.txt 2>&1 || exit 11
tail -1 $R/gpurun_out/step_prof/log.txt | cut -c1-200
