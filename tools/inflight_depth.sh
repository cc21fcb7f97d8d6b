#!/bin/bash
# GPU box: the pipelined headline with 2 vs 3 batches in flight (LLFE_INFLIGHT), alternated
# twice, after the submit/collect parity tests
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pipeline.py -k "submit or flight or empty" > gpurun_out/inflight_tests.log 2>&1 \
    || { tail -30 gpurun_out/inflight_tests.log; exit 1; }
tail -2 gpurun_out/inflight_tests.log
for d in 2 3 2 3; do
    LLFE_INFLIGHT=$d timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 \
        --e2e-host-steps 0 --per-class-steps 0 --steps ${STEPS:-10} --warmup 3 \
        > gpurun_out/inflight_$d.json 2> gpurun_out/inflight_$d.err || { tail -5 gpurun_out/inflight_$d.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/inflight_$d.json').read().strip().splitlines()[-1])
print('inflight $d: %.0f images/s, %.2f ms/step, contour busy %s' % (d['value'], d['ms_per_step'], d.get('host_contour_busy')))"
done
