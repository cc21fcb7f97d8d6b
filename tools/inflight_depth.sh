#!/bin/bash
# GPU box: the pipelined bench with 2 vs 3 batches in flight (LLFE_INFLIGHT), alternated
# twice, after the submit/collect parity tests.  Usage: tools/inflight_depth.sh TAG [bench args]
# (round 5: TAG c2 with --batch 256 --features colors,shapes = BASELINE configs[2]).
set -u -o pipefail
TAG=${1:-c3}; shift || true
O=gpurun_out/inflight_$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pipeline.py -k "submit or flight or empty" > $O/tests.log 2>&1 \
    || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for d in 2 3 2 3; do
    LLFE_INFLIGHT=$d timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 \
        --e2e-host-steps 0 --per-class-steps 0 --steps ${STEPS:-10} --warmup 3 "$@" \
        >> $O/depth_$d.json 2>> $O/depth_$d.err || { tail -5 $O/depth_$d.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$O/depth_$d.json').read().strip().splitlines()[-1])
print('inflight $d: %.0f images/s, %.2f ms/step, result assembly %s, contour busy %s' % (d['value'], d['ms_per_step'], d.get('result_assembly'), d.get('host_contour_busy')))"
done
