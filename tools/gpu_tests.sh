#!/bin/bash
# GPU box: the given test files (default: the whole -m gpu suite)
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/gpu_tests.log | tail -5
tail -30 gpurun_out/gpu_tests.log | grep -vE "PASSED" | tail -25
exit $rc
