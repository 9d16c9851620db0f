#!/bin/bash
# Round 5: full-model stage table (AANet, AANet+) + the kernel-trace stats of the AANet bench.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/fm
export PYTHONUNBUFFERED=1
for m in aanet aanetplus; do
  timeout -k 10 300 python tools/full_model_stages.py $m --iters 5 > gpurun_out/fm/stages_$m.txt 2>&1 || { tail -5 gpurun_out/fm/stages_$m.txt; exit 3; }
  grep -v "^{" gpurun_out/fm/stages_$m.txt | grep -v "Warning\|warn\|amdgpu.ids"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/fm/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --model aanet --steps 3 --warmup 1 --no-graph > $GRAFT_REPO_ROOT/gpurun_out/fm/traced.log 2>&1 || exit 4
echo traced
