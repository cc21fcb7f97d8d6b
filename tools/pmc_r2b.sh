#!/bin/bash
# GPU box: SQ counter passes (issue / wait / LDS / SALU) for k_kmeans (colours only) and
# k_stencil_stream (shapes + shadows only)
set -u -o pipefail
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
B="SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INST_CYCLES_SALU"
C="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_VMEM_WR SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_SENDMSG SQ_WAIT_INST_ANY"
bash tools/pmc.sh kmA "$A" k_kmeans --features colors --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh kmB "$B" k_kmeans --features colors --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh kmC "$C" k_kmeans --features colors --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh stA "$A" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0 &&
bash tools/pmc.sh stB "$B" k_stencil --features shapes,shadows --e2e-png-steps 0 --e2e-jpeg-steps 0
