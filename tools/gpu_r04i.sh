#!/bin/bash
# Round 4: same-call A/B of the DCN tail's tile order (base = row-major, colmaj = -DDCN_COLMAJOR=1):
# bench step + per-kernel lines, then one FETCH_SIZE / WRITE_SIZE pass of the roofline loops each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VARS=${VARS:-"base colmaj unroll"}
lib() { [ $1 = base ] && echo $R/aanet_amd/libaanet_mi355x.so || echo $R/aanet_amd/libaanet_mi355x_$1.so; }
for r in 1 2; do
  for V in $VARS; do
    AANET_MI355X_LIB=$(lib $V) timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r04i_$V.json 2>&1 || exit 8
    python -c "import json; d=json.loads(open('gpurun_out/r04i_$V.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$V', round(d['ms_per_step'],4), 'ms', 'dcn', round(k['mdcn_pw_s0']['ms']*1e3,1), 'c3', round(k['conv3x3_pw_s0']['ms']*1e3,1), 'off', round(k['offset_conv_s0']['ms']*1e3,1), 'epe', d['epe_vs_ref'])"
  done
done
cd /tmp && export TMPDIR=/tmp
for V in $VARS; do
  for C in FETCH_SIZE WRITE_SIZE; do
    AANET_MI355X_LIB=$(lib $V) timeout -k 10 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $R/gpurun_out/r04i_pmc_${V}_$C -o run -- \
      python3 $R/bench.py --only mdcn --steps 5 --warmup 1 > $R/gpurun_out/r04i_pmc_${V}_$C.log 2>&1 || exit 9
  done
done
cd $R && python tools/pmc_report.py gpurun_out/r04i_pmc_base_FETCH_SIZE dcn_tile_kernel conv_fwd_kernel conv3x3_g3 shift_volume && \
  python tools/pmc_report.py gpurun_out/r04i_pmc_colmaj_FETCH_SIZE dcn_tile_kernel && python tools/pmc_report.py gpurun_out/r04i_pmc_unroll_FETCH_SIZE dcn_tile_kernel
echo r04i done
