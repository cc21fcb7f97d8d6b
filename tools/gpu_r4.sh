#!/bin/bash
# GPU box (round 4): the whole -m gpu suite, one default bench line (CPU baseline, e2e and
# per-class legs included), then the rocprofv3 kernel-trace + PMC passes (tools/profile.sh TAG)
set -u -o pipefail
TAG=${1:-r4}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
brc=$?
head -c 1200 gpurun_out/bench_$TAG.json; echo
tail -3 gpurun_out/bench_$TAG.err
if [ $brc -ne 0 ]; then echo "bench exit $brc: stopping"; exit $brc; fi
bash tools/profile.sh $TAG
bash tools/png_split.sh || { echo "png split failed"; exit 1; }
