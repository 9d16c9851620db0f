#!/bin/bash
# Round 4: int64 fixed-point window DCN backward (16-channel slices) in both modes -- DCN tests,
# then the C4 sweep (auto = window in both modes; global-atomic leg for comparison).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mdcn.py tests/test_gpu_train.py tests/test_gpu_engine_conv.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04n_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r04n_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python bench.py --dcn-sweep --kernel-iters 10 > gpurun_out/r04n_sweep.jsonl 2> gpurun_out/r04n_sweep.err || exit 7
python -c "
import json
for l in open('gpurun_out/r04n_sweep.jsonl'):
    d=json.loads(l)
    if 'shape' in d: print(d['shape'], 'fwd %.0f bwd %.0f det %.0f global %.0f us' % (d['fwd_us'], d['bwd_us'], d['bwd_det_us'], d['bwd_global_atomic_us']))
"

if [ -n "${TRAIN:-}" ]; then
  timeout -k 10 300 python bench.py --train --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04n_train.json 2>gpurun_out/r04n_train.err || exit 13
  timeout -k 10 300 python bench.py --train --deterministic --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04n_train_det.json 2>gpurun_out/r04n_train_det.err || exit 14
  python -c "
import json
for f in ('gpurun_out/r04n_train.json', 'gpurun_out/r04n_train_det.json'):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, round(d['ms_per_step'], 3), 'ms', round(d['value'], 1), 'pairs/s')
"
fi
exit $rc
