#!/bin/bash
# Round 5 first pass: split exactness probe, the tests the RNE split / NaN poison / near-tie
# bound / window forward touch, the C4 forward at agg_s0/s1, then the bench-step A/B against
# abl/libold.so (truncation split).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/split_rne_lab || exit 3
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_split.py tests/test_gpu_dcn_tile.py tests/test_gpu_mdcn.py tests/test_gpu_models.py \
  tests/test_gpu_production.py > gpurun_out/pytest_r05a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r05a.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --dcn-sweep --dcn-shapes agg_s0,agg_s1 --kernel-iters 10 > gpurun_out/sweep_r05a.jsonl 2>&1 || exit 6
python -c "
import json
for l in open('gpurun_out/sweep_r05a.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        if 'shape' in d: print(d['shape'], 'fwd %.1f us (window %s) generic %.1f us bwd %.1f det %.1f' % (d['fwd_us'], d['fwd_window'], d['fwd_generic_us'], d['bwd_us'], d['bwd_det_us']))
"
bash tools/ab_step.sh || exit 5
exit $rc
