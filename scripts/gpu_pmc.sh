#!/bin/bash
# gpu_pmc.sh TAG -- latency variants of the level kernel (onewg.sh) and PMC
# passes over scripts/kbench.py, one counter group per pass.
set -e -o pipefail
TAG=$1
R=$(pwd)
bash "$R/scripts/onewg.sh" "$TAG"
cd "$R"
bash "$R/scripts/pmc_sweep.sh" "$TAG" \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
  "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" \
  "FETCH_SIZE" "WRITE_SIZE"
echo "pmc $TAG done"
