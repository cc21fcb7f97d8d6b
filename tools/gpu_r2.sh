#!/bin/bash
# GPU box: full GPU test suite then one default bench line (no CPU baseline)
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py --cpu-baseline off "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json | head -c 1500; echo
tail -3 gpurun_out/bench.err
exit $brc
