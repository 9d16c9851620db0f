#!/bin/bash
# Same-call A/B of the DCN backward (C4 sweep, agg_s0 / agg_s1) between abl/libold.so and the
# in-tree build, after the DCN GPU tests.  Usage: bash tools/ab_dcn_bwd.sh
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mdcn.py tests/test_gpu_train.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 3; }
tail -1 gpurun_out/ab_tests.log
for i in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export AANET_MI355X_LIB=$PWD/abl/libold.so; else unset AANET_MI355X_LIB; fi
    timeout -k 10 200 python bench.py --dcn-sweep --dcn-shapes agg_s0,agg_s1 --kernel-iters 10 > gpurun_out/ab_sweep_$v.jsonl 2>/dev/null || exit 4
    python -c "
import json
for l in open('gpurun_out/ab_sweep_$v.jsonl'):
    d=json.loads(l)
    if 'shape' in d: print('$v', d['shape'], 'bwd %.0f det %.0f us' % (d['bwd_us'], d['bwd_det_us']))
"
  done
done
