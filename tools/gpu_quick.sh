#!/bin/bash
# Quick GPU loop: GPU tests (all, or PYTEST_K subset), microbench cases, one bench line.
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ -n "${MB:-}" ] && { timeout -k 5 120 python tools/conv_microbench.py 20 $MB || exit $?; }
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit $?
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 3), "epe", d["epe_vs_ref"], "max", d["max_abs_disp_err_vs_ref"])
for k, v in d["kernels"].items(): print(" ", k, round(v["ms"] * 1e3, 1), "us frac", round(v["frac"], 3))
PY
exit $rc
