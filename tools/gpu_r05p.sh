#!/bin/bash
# Offset conv (conv_g3) VALU trims: its tests, then a same-call A/B of the bench step against
# abl/libg3a.so (offset_conv_s0 / conv3x3_pw_s0 / mdcn_pw_s0 live times).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_g3.py tests/test_gpu_production.py tests/test_gpu_models.py tests/test_gpu_conv.py tests/test_gpu_engine_conv.py tests/test_gpu_split.py > gpurun_out/r05p_pytest.txt 2>&1 || { tail -20 gpurun_out/r05p_pytest.txt; exit 3; }
tail -1 gpurun_out/r05p_pytest.txt
for r in 1 2; do
for L in aanet_amd/libaanet_mi355x.so abl/libg3a.so; do
  AANET_MI355X_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null > gpurun_out/ab_lib.json || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/ab_lib.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$L', round(d['ms_per_step'],4), 'ms/step;', '; '.join('%s %.1f us %.3f' % (n, k[n]['ms']*1e3, k[n]['frac']) for n in ('offset_conv_s0','conv3x3_pw_s0','mdcn_pw_s0') if n in k))"
done
done
