#!/bin/bash
# GPU box (round 5): k_uq_part reading each group of 8 runs as one flattened list (NF loads
# in flight): identity vs round 4's kernels, then isolated kernel times per variant.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5s_identity.log 2>&1; rc=$?; cat gpurun_out/r5s_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5s_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh
