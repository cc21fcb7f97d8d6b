#!/bin/bash
# GPU box (round 5): tile-flag hysteresis with the list loop at 62 VGPRs: identity, isolated
# times per variant, per-class kernel traces.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5w_identity.log 2>&1; rc=$?; cat gpurun_out/r5w_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5w_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
rm -f gpurun_out/r5t/summary.txt
timeout -k 10 900 bash tools/debug/cmd_r5t.sh r_seg216 f1_tflag f2_tflag f3_tflag
