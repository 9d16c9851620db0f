#!/bin/bash
# GPU session helper: parity tests, then a short bench.  Stops at the first crash/timeout
# (exit codes other than 0/1 from pytest), as the pool's rules require.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu -q ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest crashed/timed out rc=$rc"; exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.log 2>&1
brc=$?
tail -5 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
