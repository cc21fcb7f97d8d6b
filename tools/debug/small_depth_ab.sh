#!/bin/bash
# GPU box (round 6): 2 vs 3 batches in flight on the smaller configs (256 x 1080p colours,
# colours + shapes; 64 x 512^2 colours), interleaved, twice each
set -u -o pipefail
mkdir -p gpurun_out
B="python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --batcher-steps 0"
for rep in 1 2; do
for cfg in "c1:--batch 256 --features colors" "c2:--batch 256 --features colors,shapes" "c0:--batch 64 --height 512 --width 512 --features colors"; do
for d in 2 3; do
    n=${cfg%%:*}; a=${cfg#*:}
    timeout -k 10 300 $B $a --inflight $d > gpurun_out/sd_${n}_${d}.json 2> gpurun_out/sd_${n}_${d}.err || { tail -20 gpurun_out/sd_${n}_${d}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/sd_${n}_${d}.json').read().strip().splitlines()[-1])
print('$n inflight $d value %.0f ms/step %.3f' % (d['value'], d['ms_per_step']))"
done
done
done
