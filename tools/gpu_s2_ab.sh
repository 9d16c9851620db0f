cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export PYTHONUNBUFFERED=1
AANET_S2_ROWS=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_s2.py > gpurun_out/s2_tests2.log 2>&1 || { tail -20 gpurun_out/s2_tests2.log; exit 1; }
tail -1 gpurun_out/s2_tests2.log
for f in 1 2 1 2; do AANET_S2_ROWS=$f timeout -k 10 120 python tools/s2_bench.py | sed "s/^/rows=$f /" || exit 1; done
for f in 2 1; do AANET_S2_ROWS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$f.log 2>&1 || exit 1; python -c "import json; d=json.loads(open('gpurun_out/bench_$f.log').read().strip().splitlines()[-1]); print('rows=$f bench', round(d['ms_per_step'],4), d['config']['schedule'])"; done
BENCH_ARGS="--only step --steps 8 --warmup 3 --no-graph --no-cpu-baseline" PROF_TIMEOUT=240 bash tools/profile_step.sh > /dev/null 2>&1 && python tools/step_breakdown.py $(find gpurun_out/prof_step -name "*kernel_trace.csv" | head -1) -v > gpurun_out/step_bd.txt
