#!/bin/bash
# Time attribution of the window DCN tail (dcn_tile_kernel<2,32>, C2 scale 0, B=8) from the
# debug build's switches (tools/build_variant.sh dbg "-DAANET_DEBUG_SWITCHES"; AANET_DCN_DBG bits:
# 1 no MFMAs, 2 window corner reads at position 0, 4 no global fallback, 8 no per-chunk barrier,
# 16 no identity / CSA terms in the epilogue, 32 no window loads, 64 no weight DMA).  Outputs of
# a switched run are INVALID; only the time is meaningful.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
for d in 0 1 2 8 16 32 64 3 17; do
  echo "AANET_DCN_DBG=$d"
  AANET_MI355X_LIB=$R/aanet_amd/libaanet_mi355x_dbg.so AANET_DCN_DBG=$d timeout -k 10 120 \
    python3 $R/tools/dcn_tile_bench.py 20 0.5 2>&1 | grep "offset bias" || exit 1
done
