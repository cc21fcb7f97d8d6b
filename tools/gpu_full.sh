#!/bin/bash
# GPU box: GPU test suite, one default bench line (CPU baseline included), then the
# rocprofv3 kernel-trace + PMC traffic profile (tools/profile.sh TAG).
set -u -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
brc=$?
head -c 3000 gpurun_out/bench_$TAG.json; echo
tail -3 gpurun_out/bench_$TAG.err
if [ $brc -ne 0 ]; then echo "bench exit $brc: stopping"; exit $brc; fi
bash tools/profile.sh $TAG
