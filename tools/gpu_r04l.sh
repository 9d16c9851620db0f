#!/bin/bash
# Round 4: concat/difference band kernel with per-thread slots -- bit-exact tests, then the bench
# line's concat_volume_c5 and a PMC pass over the roofline loops.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_modules.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04l_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04l_bench.json 2>&1 || exit 8
  python -c "import json; d=json.loads(open('gpurun_out/r04l_bench.json').read().strip().splitlines()[-1]); k=d['kernels']['concat_volume_c5']; print('step', round(d['ms_per_step'],4), 'concat', round(k['ms']*1e3,1), 'us frac', round(k['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace --output-format csv -d $R/gpurun_out/r04l_pmc -o run -- python3 $R/bench.py --only mdcn --steps 3 --warmup 1 > $R/gpurun_out/r04l_pmc.log 2>&1 || exit 9
cd $R && python tools/pmc_report.py gpurun_out/r04l_pmc shift_volume_band
