#!/bin/bash
# Round 4: the halo form of the grouped offset conv (conv_g3.hip): its tests and timing against the
# engine's halo form, the step with it on / off (AANET_OFFSET_KERNEL), then the whole GPU suite
# (without -x), smoke and the default bench line.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_conv_g3.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04c_g3.log 2>&1
rc=$?; tail -3 gpurun_out/r04c_g3.log; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do $T 120 python tools/g3_bench.py || exit 6; done
for r in 1 2; do
  for f in 0 1; do
    AANET_OFFSET_KERNEL=$f $T 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04c_bench_$f.json 2>&1 || exit 8
    python -c "import json; d=json.loads(open('gpurun_out/r04c_bench_$f.json').read().strip().splitlines()[-1]); print('offset_kernel=$f', round(d['ms_per_step'],4), 'ms', d['config']['schedule'], 'epe', d['epe_vs_ref'], d['max_abs_disp_err_vs_ref'])"
  done
done
bash tools/gpu_full.sh
