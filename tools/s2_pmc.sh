#!/bin/bash
# Counter passes over the stride-2 heads launch (tools/s2_bench.py heads): pipe, stall, texture
# and memory counters.  S2_PASSES=short: the first four passes only.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python tools/s2_bench.py > gpurun_out/s2_bench.txt 2>&1
tail -1 gpurun_out/s2_bench.txt
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS"
P3="TA_BUSY_avr TA_BUSY_max TA_BUFFER_READ_WAVEFRONTS GRBM_GUI_ACTIVE"
P4="TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
P5="TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_LDS_BANK_CONFLICT"
if [ "${S2_PASSES:-}" = short ]; then
  PMC_NAME=${PMC_NAME:-pmc_s2} PMC_CMD="$GRAFT_REPO_ROOT/tools/s2_bench.py heads" bash tools/pmc.sh "$P1" "$P2" "$P3" "$P4"
else
  PMC_NAME=${PMC_NAME:-pmc_s2} PMC_CMD="$GRAFT_REPO_ROOT/tools/s2_bench.py heads" bash tools/pmc.sh "$P1" "$P2" "$P3" "$P4" "$P5" \
    "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_SALU"
fi
