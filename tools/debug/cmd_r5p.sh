#!/bin/bash
# GPU box (round 5): parameter sweep of the final build (stencil segment rows, k-means push
# unroll, k-means++ chunk runs): isolated kernel times and the pipelined headline per
# variant; then the base build with three batches in flight.
set -u -o pipefail
mkdir -p gpurun_out/r5p
export TMPDIR=/tmp
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
echo "pipelined:"; timeout -k 10 700 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 || exit 1
for d in 3 2; do
    LLFE_INFLIGHT=$d timeout -k 10 240 python bench.py --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 \
        --per-class-steps 0 > gpurun_out/r5p/inflight$d.json 2> gpurun_out/r5p/inflight$d.err || { tail -5 gpurun_out/r5p/inflight$d.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/r5p/inflight$d.json').read().strip().splitlines()[-1]); print('inflight $d', d['value'], d['ms_per_step'], d.get('inflight'))"
done
