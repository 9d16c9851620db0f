#!/bin/bash
# Round 4, part 1: offset conv halo kernel + atomic-free window DCN backward: tests and timing.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_conv_g3.py tests/test_gpu_mdcn.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04e_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r04e_tests.log; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do $T 100 python tools/g3_bench.py || exit 6; done
$T 200 python bench.py --dcn-sweep --kernel-iters 10 > gpurun_out/r04e_sweep.jsonl 2> gpurun_out/r04e_sweep.err || exit 7
python -c "
import json
for l in open('gpurun_out/r04e_sweep.jsonl'):
    d=json.loads(l)
    if 'shape' in d: print(d['shape'], 'fwd %.0f bwd %.0f det %.0f global %.0f us' % (d['fwd_us'], d['bwd_us'], d['bwd_det_us'], d['bwd_global_atomic_us']))
"
exit $rc
