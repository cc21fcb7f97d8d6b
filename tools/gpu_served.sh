#!/bin/bash
# GPU box: the served-launch parity tests (tests/test_gpu_served.py) and the given extra
# test selections, progress in gpurun_out/served.log
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_served.py "$@" -m gpu -x -v -s --timeout 900 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/served.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|served" gpurun_out/served.log | tail -40
tail -40 gpurun_out/served.log | grep -vE "PASSED|\[served" | tail -30
exit $rc
