#!/bin/bash
# Round 5: the pipelined window DCN kernel (dcn_win.hip) -- split probe, the window / split /
# production / DCN tests, then a same-call A/B of the DCN tail alone and the bench step:
# in-tree (dcn_win), abl/libold.so (round-4 kernel), both with the truncation split;
# then the C4 forward at agg_s0/s1.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 60 ./tools/split_rne_lab || exit 3
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dcn_tile.py tests/test_gpu_split.py tests/test_gpu_mdcn.py tests/test_gpu_production.py \
  tests/test_gpu_models.py > gpurun_out/pytest_r05b.log 2>&1
rc=$?; tail -8 gpurun_out/pytest_r05b.log; [ $rc -le 1 ] || exit $rc
ROUNDS=2 bash tools/ab_libs.sh $PWD/aanet_amd/libaanet_mi355x.so $PWD/abl/libold.so $PWD/abl/libprio.so || exit 5
for L in aanet_amd/libaanet_mi355x.so abl/libold.so; do
AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --dcn-sweep --dcn-shapes agg_s0,agg_s1 --kernel-iters 10 > gpurun_out/sweep_r05b.jsonl 2>&1 || exit 6
echo "== $L"
python -c "
import json
for l in open('gpurun_out/sweep_r05b.jsonl'):
    if l.startswith('{'):
        d = json.loads(l)
        if 'shape' in d: print(d['shape'], 'fwd %.1f us (window %s) generic %.1f us bwd %.1f det %.1f' % (d['fwd_us'], d['fwd_window'], d['fwd_generic_us'], d['bwd_us'], d['bwd_det_us']))
"
done
exit $rc
