#!/bin/bash
# GPU box (round 6): served_batcher with 2 vs 3 launches in flight (MicroBatcher inflight),
# beside the headline of the same run, interleaved, twice each
set -u -o pipefail
mkdir -p gpurun_out
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 ${BD_ARGS:-}"
for rep in 1 2; do
for d in 2 3; do
    timeout -k 10 300 python bench.py $ARGS --batcher-inflight $d > gpurun_out/bd_$d.json 2> gpurun_out/bd_$d.err || { tail -20 gpurun_out/bd_$d.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/bd_$d.json').read().strip().splitlines()[-1]); b=d['served_batcher']
print('batcher inflight $d value %.0f served %.0f ratio %.3f worker %s' % (d['value'], b['value'], b['value'] / d['value'], b['worker']))"
done
done
