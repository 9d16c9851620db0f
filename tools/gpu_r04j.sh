#!/bin/bash
# Round 4: FETCH_SIZE calibration of 64-B segment reads (tools/fetch_calib.hip) and the offset
# conv's pipe/LDS counters (g3_bench).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/calib
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/calib/f -o run -- $R/tools/fetch_calib > $R/gpurun_out/calib/f.log 2>&1 || exit 3
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace --output-format csv -d $R/gpurun_out/calib/r -o run -- $R/tools/fetch_calib > $R/gpurun_out/calib/r.log 2>&1 || echo "rdreq pass failed (counter names)"
cd $R && python tools/pmc_report.py gpurun_out/calib k_ || exit 4
cd $R && PMC_NAME=pmc_g3 PMC_CMD="$R/tools/g3_bench.py" bash tools/pmc.sh \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_INSTS_LDS" \
  "SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL" || exit 5
python tools/pmc_report.py gpurun_out/pmc_g3 conv3x3_g3_kernel
echo r04j done
