#!/bin/bash
# GPU box (round 5): hysteresis over the stencil's flagged tiles only (tile flags + a
# list-driven k_ccl_local): identity vs round 4's kernels, isolated times per variant,
# per-class kernel traces, then the GPU tests with the in-tree build.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 bash tools/debug/cmd_r5t.sh r_seg216 e_tflag || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5u_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5u_tests.log; exit $rc
