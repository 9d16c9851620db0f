#!/bin/bash
# conv2d_wgrad default = fixed-order partials: engine-conv and training tests, then the training
# step (float and deterministic) and its kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/train_prof2
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_engine_conv.py tests/test_gpu_train.py 2>&1 | tail -3 || exit 1
timeout -k 10 300 python bench.py --train --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1 > gpurun_out/train_float2.json || exit 2
cat gpurun_out/train_float2.json
timeout -k 10 300 python bench.py --train --deterministic --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | tail -1 > gpurun_out/train_det2.json || exit 3
cat gpurun_out/train_det2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/train_prof2 -o tr -- \
  python3 $R/bench.py --train --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/train_prof2/log.txt 2>&1 || exit 11
echo done
