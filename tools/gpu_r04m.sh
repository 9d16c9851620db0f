#!/bin/bash
# Round 4: write-bandwidth probe variants, then the concat band kernel with plain (base) vs
# non-temporal (cvnt build) stores, same call.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
[ -n "${PROBE:-}" ] && { timeout -k 10 60 ./tools/write_ceiling || exit 3; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -rf --timeout 120 --timeout-method thread -k "concat or diff or shift or volume" > gpurun_out/r04m_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r04m_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2; do
  for V in ${VARS:-base ds2 ds4 yb4}; do
    L=aanet_amd/libaanet_mi355x_$V.so; [ $V = base ] && L=aanet_amd/libaanet_mi355x.so
    AANET_MI355X_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04m_$V.json 2>&1 || exit 8
    python -c "import json; d=json.loads(open('gpurun_out/r04m_$V.json').read().strip().splitlines()[-1]); k=d['kernels']['concat_volume_c5']; print('$V step', round(d['ms_per_step'],4), 'concat', round(k['ms']*1e3,1), 'us frac', round(k['frac'],3))"
  done
done
