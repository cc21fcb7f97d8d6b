#!/bin/bash
# GPU box (round 5): the hysteresis list passes (border, flatten, strong, edge) with 16k /
# 64k workgroups instead of 4096 looping over the listed tiles: parity subset, identity,
# isolated times, per-class traces.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 60 --timeout-method thread -k "canny or shape_mask or dilate" > gpurun_out/r5aj_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r5aj_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5aj_identity.log 2>&1; rc=$?; cat gpurun_out/r5aj_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5aj_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
rm -f gpurun_out/r5t/summary.txt
timeout -k 10 900 bash tools/debug/cmd_r5t.sh k_final s_grid16384 s_grid65536 || exit 1
