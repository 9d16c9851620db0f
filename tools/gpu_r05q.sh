#!/bin/bash
# DCN tail: offset statistics vs time (window kernel vs generic engine), and the debug build's
# attribution of the out-of-window fallback (AANET_DCN_DBG=4 skips it: outputs invalid).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/dcn_tile_bench.py 20 0,0.5,1.0 || exit 3
for d in 0 4; do
  echo "== debug build AANET_DCN_DBG=$d"
  AANET_DCN_DBG=$d AANET_MI355X_LIB=$PWD/abl/libdbg.so timeout -k 10 200 python tools/dcn_tile_bench.py 20 0,0.5,1.0 2>&1 | grep -v "^aanet:" || exit 4
done
