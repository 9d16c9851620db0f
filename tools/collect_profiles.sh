#!/bin/bash
# Round profile collection: (1) kernel-trace + stats of the default bench command,
# (2) separate PMC passes (FETCH_SIZE / WRITE_SIZE, SQ counters) over the per-kernel roofline loop.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02}
OUT=$R/gpurun_out/profiles_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_traced.log 2>&1 || exit $?
i=0
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- \
    python3 $R/bench.py --only mdcn --steps 5 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo collected
