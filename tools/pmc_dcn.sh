#!/bin/bash
# Counter passes over one conv_microbench case (default: the scale-0 DCN tail with CSA).
# Usage: bash tools/pmc_dcn.sh [case]  -> gpurun_out/pmc_dcn/ ; summarise with tools/pmc_report.py
CASE=${1:-dcn_pw_nhwc_csa}
PMC_NAME=pmc_dcn PMC_CMD="${GRAFT_REPO_ROOT:-$(pwd)}/tools/conv_microbench.py 5 $CASE" bash tools/pmc.sh \
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
 "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS" \
 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" \
 "FETCH_SIZE" "WRITE_SIZE"
