# GPU box helper: a test subset, then the step kernel traces (serial and concurrent schedules).
# usage: bash tools/gpu_round.sh "<pytest -k / file args>"
set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $1 > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
  tail -3 gpurun_out/tests.log
fi
for cfg in "0 1" "1 1"; do
  set -- $cfg
  tag=cs$1_pf$2
  AANET_CONCURRENT_SCALES=$1 AANET_POST_FUSION=$2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --only step --steps 8 --warmup 3 --no-graph --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --kernel-iters 20 > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log | cut -c1-400
