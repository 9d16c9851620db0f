#!/bin/bash
# Full verification: every GPU test WITHOUT -x (one failure cannot hide the rest), smoke(), then
# one default bench line.  A test failure (rc 1) continues to smoke/bench; a fault, abort or
# time limit stops the script.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rfs --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 4; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_full.json 2>&1 || exit 5
python -c "import json; d=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],1), 'pairs/s', round(d['ms_per_step'],4), 'ms', d['config']['schedule'], 'roof', d['roofline']['kernel'], round(d['roofline']['frac'],3), 'epe', d['epe_vs_ref'])"
exit $rc
