#!/bin/bash
# GPU box: SQ counter passes for k_stencil (shapes+shadows only) and k_kmeans (colours only)
set -u -o pipefail
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
B="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_SALU"
bash tools/pmc.sh stA "$A" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh stB "$B" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh kmA "$A" k_kmeans --features colors --e2e-png-steps 0 --e2e-jpeg-steps 0
