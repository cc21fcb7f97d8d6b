#!/bin/bash
# GPU box (round 6): identity, the GPU tests of one file pattern (-k), then served A/B
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/q_identity.log 2>&1; rc=$?; cat gpurun_out/q_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/q_identity.log && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "${TESTK:-batcher}" > gpurun_out/q_tests.log 2>&1
rc=$?; tail -4 gpurun_out/q_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/debug/served_ab.sh
