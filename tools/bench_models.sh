#!/bin/bash
# Headline bench + full-model benches (+ kernel traces of the full models).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${OUT_NAME:-models}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/headline.json 2> $OUT/headline.err || exit $?
for m in aanet aanetplus; do
  timeout -k 10 300 python3 $R/bench.py --model $m --steps 10 --warmup 3 > $OUT/$m.json 2> $OUT/$m.err || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$m -o run -- \
    python3 $R/bench.py --model $m --steps 3 --warmup 1 --no-graph > $OUT/${m}_traced.log 2>&1 || exit $?
done
cat $OUT/headline.json $OUT/aanet.json $OUT/aanetplus.json
