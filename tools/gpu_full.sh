#!/bin/bash
# Full verification: every GPU test, smoke(), then one default bench line.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2>&1 || exit 1
python -c "import json; d=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],4), 'ms', d['config']['schedule'], 'roof', d['roofline']['kernel'], round(d['roofline']['frac'],3), 'epe', d['epe_vs_ref'])"
