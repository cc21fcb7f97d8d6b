#!/bin/bash
# GPU box (round 5 final): identity vs round 4's kernels, then tools/gpu_r5.sh r5ak (GPU
# tests, default bench, rocprofv3 kernel trace + PMC passes).
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5ak_identity.log 2>&1; rc=$?; cat gpurun_out/r5ak_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5ak_identity.log && exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5ak_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r5ak_smoke.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_r5.sh r5ak
