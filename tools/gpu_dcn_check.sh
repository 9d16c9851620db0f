set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dcn_tile.py tests/test_gpu_split.py tests/test_gpu_production.py > gpurun_out/t_dcn.log 2>&1
rc=$?; tail -25 gpurun_out/t_dcn.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench2.log 2>&1
rc=$?; tail -3 gpurun_out/bench2.log; exit $rc
