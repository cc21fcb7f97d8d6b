#!/bin/bash
# GPU box (round 6): the headline with 2 vs 3 batches in flight, interleaved, twice each
set -u -o pipefail
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --batcher-steps 0"
for rep in 1 2; do
for d in 2 3; do
    timeout -k 10 300 python bench.py $ARGS --inflight $d > gpurun_out/if_$d.json 2> gpurun_out/if_$d.err || { tail -20 gpurun_out/if_$d.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/if_$d.json').read().strip().splitlines()[-1])
print('inflight $d value %.0f ms/step %.2f one-at-a-time %s serving %s' % (d['value'], d['ms_per_step'], d['value_one_batch_at_a_time'], d.get('serving_thread')))"
done
done
