#!/bin/bash
# SQ counter passes over the bior1.5 op (per kernel): issue / wait / LDS / memory-instruction mix.
#   bash tools/wl_pmc.sh <out_dir> [op]
set -u
bash tools/pmc_pass.sh "${1:-wl_pmc}" "${2:-wavelet_bior15}" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
