#!/bin/bash
# GPU box: SQ counter passes for k_stencil* (shapes+shadows only)
set -u -o pipefail
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
B="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS"
bash tools/pmc.sh ${1}A "$A" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh ${1}B "$B" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0
