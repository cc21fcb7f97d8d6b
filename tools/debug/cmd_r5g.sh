#!/bin/bash
# GPU box (round 5): identity of the stencil candidate fix (+ k-means++ selection forms),
# the GPU test suite on it, the pipelined timeline, variant timings, and the headline with
# more HIP hardware queues.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5g_identity.log 2>&1; echo "identity rc=$?"; cat gpurun_out/r5g_identity.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r5g_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 300 python tools/debug/pipe_timeline.py gpurun_out/r5g_pipe2.txt 8 2 > gpurun_out/r5g_pipe2.log 2>&1 || { tail -20 gpurun_out/r5g_pipe2.log; exit 1; }
cat gpurun_out/r5g_pipe2.log
timeout -k 10 600 bash tools/debug/run_variants.sh || exit 1
echo "pipelined:"; timeout -k 10 600 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 || exit 1
echo "GPU_MAX_HW_QUEUES=8:"; GPU_MAX_HW_QUEUES=8 timeout -k 10 300 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 || exit 1
