#!/bin/bash
# Round 4 profiles: bench kernel stats + PMC passes (profiles/r04_*), the SURVEY C4 DCN sweep,
# and pipe/LDS counter passes of the offset conv (g3_bench).  Each step has its own time limit.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=r04 bash tools/collect_profiles.sh || exit 11
cd $R && bash tools/c4_sweep.sh || exit 12
cd $R && PMC_NAME=pmc_g3 PMC_CMD="$R/tools/g3_bench.py" bash tools/pmc.sh \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS" \
  "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" || exit 13
echo r04h done
