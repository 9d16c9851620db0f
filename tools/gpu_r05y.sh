#!/bin/bash
# Training step at HEAD: bench.py --train float and deterministic lines, then the rocprofv3
# kernel trace of the float step for tools/train_breakdown.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/train_prof
cd $R
timeout -k 10 300 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1 > gpurun_out/train_float.json || exit 1
cat gpurun_out/train_float.json
timeout -k 10 300 python bench.py --train --deterministic --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1 > gpurun_out/train_det.json || exit 2
cat gpurun_out/train_det.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/train_prof -o tr -- \
  python3 $R/bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/train_prof/log.txt 2>&1 || exit 11
tail -1 $R/gpurun_out/train_prof/log.txt
echo done
