#!/bin/bash
# GPU box (round 5): the pipelined headline and 12-step per-class lines of round 4's kernels
# (a), the r5r commit (p) and the final build (k), twice each, to tell the per-class ui
# change from run-to-run noise.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
    timeout -k 10 900 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 --per-class-steps 12 || exit 1
done
