#!/bin/bash
# GPU-box check: parity tests, then (only if the tests ran to completion without a
# crash/timeout) one bench line.  Outputs under gpurun_out/.
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json
tail -5 gpurun_out/bench.err
[ $brc -ne 0 ] && exit $brc
exit $rc
