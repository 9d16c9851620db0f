#!/bin/bash
# deform_conv2d forward + backward microbench over the aggregation / feature DCN
# shapes (bench.py --dcn-sweep), its kernel-trace stats, and PMC passes (MFMA/VALU issue, MFMA
# busy cycles, HBM traffic) per kernel.  Output: gpurun_out/c4/ ; summary: tools/c4_summary.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/c4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/bench.py --dcn-sweep --kernel-iters 10 > $OUT/sweep.jsonl 2>$OUT/sweep.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c4 -- \
  python3 $R/bench.py --dcn-sweep --kernel-iters 3 > $OUT/trace.log 2>&1 || exit $?
i=0
for pass in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- \
    python3 $R/bench.py --dcn-sweep --kernel-iters 2 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
done
echo c4 collected
