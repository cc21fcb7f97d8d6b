#!/bin/bash
# GPU box (round 5): the GPU test suite, the default bench line, and the rocprofv3
# kernel-trace + PMC passes of tools/profile.sh (TAG = $1).
set -u -o pipefail
TAG=${1:-r5}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -6 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_bench.json
timeout -k 10 1200 bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
tail -40 gpurun_out/${TAG}_profile.log
