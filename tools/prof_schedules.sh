set -e
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for cfg in "1 1" "0 1" "1 0"; do
  set -- $cfg
  tag=cs$1_pf$2
  AANET_CONCURRENT_SCALES=$1 AANET_POST_FUSION=$2 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --only step --steps 8 --warmup 3 --no-graph --no-cpu-baseline > gpurun_out/prof_$tag.log 2>&1
  tail -2 gpurun_out/prof_$tag.log
done
