#!/bin/bash
# Round 4: timing attribution of the window DCN backward at agg_s0 (debug build: AANET_DCN_BWD_DBG
# 1 = no grad_x scatter and no flush, 2 = no flush; results INVALID) + a kernel trace.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
for D in 0 1 2; do :;
  AANET_MI355X_LIB=aanet_amd/libaanet_mi355x_dbg.so AANET_DCN_BWD_DBG=$D timeout -k 10 200 python bench.py --dcn-sweep --dcn-shapes agg_s0 --kernel-iters 10 > gpurun_out/r04o_$D.jsonl 2>/dev/null || exit 7
  python -c "
import json
for l in open('gpurun_out/r04o_$D.jsonl'):
    d=json.loads(l)
    if 'shape' in d: print('dbg $D', d['shape'], 'bwd %.0f det %.0f global %.0f us' % (d['bwd_us'], d['bwd_det_us'], d['bwd_global_atomic_us']))
"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r04o_trace -o t -- python3 $R/bench.py --dcn-sweep --dcn-shapes agg_s0 --kernel-iters 3 > $R/gpurun_out/r04o_trace.log 2>&1 || exit 8
cd $R && python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04o_trace/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:90]}")
PY
