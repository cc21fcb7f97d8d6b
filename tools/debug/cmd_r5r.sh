#!/bin/bash
# GPU box (round 5): identity of the current build vs round 4's kernels, then tests + default
# bench + rocprof / PMC profile (tools/gpu_r5.sh r5r).
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5r_identity.log 2>&1; rc=$?; cat gpurun_out/r5r_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5r_identity.log && exit 1
bash tools/gpu_r5.sh r5r
