#!/bin/bash
# GPU box (round 5): tests + default bench + rocprof/PMC profile of the current tree, then
# the stencil's SQ counters per synthetic class.
set -u -o pipefail
bash tools/gpu_r5.sh r5i || exit 1
timeout -k 10 400 bash tools/debug/stencil_pmc_kind.sh > gpurun_out/r5i_spk.log 2>&1 || { echo "stencil pmc failed"; tail -20 gpurun_out/r5i_spk.log; exit 1; }
cat gpurun_out/stencil_pmc_kind/summary.txt
