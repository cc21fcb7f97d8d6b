#!/bin/bash
# GPU box (round 5): stencil segment rows (LLFE_ST_SEG) sweep after the candidate-lane fix:
# isolated kernel times and the pipelined headline per variant.
set -u -o pipefail
mkdir -p gpurun_out/r5q
export TMPDIR=/tmp
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
echo "pipelined:"; timeout -k 10 700 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 || exit 1
