#!/bin/bash
# rocprofv3 kernel trace of the deterministic training step (bench.py --train --deterministic).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/train_det_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/train_det_prof -o tr -- \
  python3 $R/bench.py --train --deterministic --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/train_det_prof/log.txt 2>&1 || exit 11
tail -1 $R/gpurun_out/train_det_prof/log.txt
echo done
