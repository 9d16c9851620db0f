#!/bin/bash
# Flakiness check: the DCN / production / model GPU tests twice in a row (separate processes).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dcn_tile.py tests/test_gpu_production.py tests/test_gpu_models.py tests/test_gpu_mdcn.py > gpurun_out/r05s_$r.txt 2>&1
  rc=$?; echo "run $r rc=$rc: $(tail -1 gpurun_out/r05s_$r.txt)"; grep "^FAILED" gpurun_out/r05s_$r.txt
  [ $rc -le 1 ] || exit $rc
done
