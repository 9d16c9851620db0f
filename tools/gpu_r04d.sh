#!/bin/bash
# Round 4: the offset conv halo kernel (conv_g3.hip) and the atomic-free window DCN backward:
# their tests, timing A/Bs, then the whole GPU suite, smoke and the default bench line.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_gpu_conv_g3.py tests/test_gpu_mdcn.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1
rc=$?; tail -6 gpurun_out/r04d_tests.log; [ $rc -le 1 ] || exit $rc
for r in 1 2 3; do $T 120 python tools/g3_bench.py || exit 6; done
$T 300 python bench.py --dcn-sweep --kernel-iters 10 > gpurun_out/r04d_sweep.jsonl 2> gpurun_out/r04d_sweep.err || exit 7
python -c "
import json
for l in open('gpurun_out/r04d_sweep.jsonl'):
    d=json.loads(l)
    if 'shape' in d: print(d['shape'], 'fwd %.0f bwd %.0f det %.0f global %.0f us' % (d['fwd_us'], d['bwd_us'], d['bwd_det_us'], d['bwd_global_atomic_us']))
"
for r in 1 2; do
  for f in 0 1; do
    AANET_OFFSET_KERNEL=$f $T 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04d_bench_$f.json 2>&1 || exit 8
    python -c "import json; d=json.loads(open('gpurun_out/r04d_bench_$f.json').read().strip().splitlines()[-1]); print('offset_kernel=$f', round(d['ms_per_step'],4), 'ms', d['config']['schedule'], 'epe', d['epe_vs_ref'], d['max_abs_disp_err_vs_ref'])"
  done
done
# DCN tail variants (tools/build_variant.sh: DCN_NOOK, DCN_NT): parity, then same-call timing
for V in nook nt ntnook lb2 prio pf pfnook; do
  AANET_MI355X_LIB=aanet_amd/libaanet_mi355x_$V.so $T 300 python -u -m pytest tests/test_gpu_dcn_tile.py tests/test_gpu_split.py -m gpu -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04d_tests_$V.log 2>&1
  rc2=$?; echo "== $V tests"; tail -2 gpurun_out/r04d_tests_$V.log; [ $rc2 -le 1 ] || exit $rc2
done
for r in 1 2 3; do
  for V in base nook nt ntnook lb2 prio pf pfnook; do
    L=aanet_amd/libaanet_mi355x_$V.so; [ $V = base ] && L=aanet_amd/libaanet_mi355x.so
    echo "== $V round $r"; AANET_MI355X_LIB=$L $T 120 python tools/dcn_tile_bench.py 30 0.5 || exit 9
  done
done
bash tools/gpu_full.sh
