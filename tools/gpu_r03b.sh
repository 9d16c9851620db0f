#!/bin/bash
# Round-3 mid-session record: bench A/B of the narrow stride-2 row form, the default bench line,
# the offset-conv microbenchmark, then the profile collection (kernel stats + PMC passes).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do for f in 1 2; do
  AANET_S2_ROWS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --kernel-iters 5 > gpurun_out/ab_rows_$f.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_rows_$f.log').read().strip().splitlines()[-1]); print('rows=$f', round(d['ms_per_step'],4), d['config']['schedule'])"
done; done
timeout -k 10 120 python tools/g3_bench.py || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r03b.json 2>&1 || exit 1
tail -c 300 gpurun_out/bench_r03b.json
TAG=r03b bash tools/collect_profiles.sh
