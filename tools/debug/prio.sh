#!/bin/bash
# GPU box: the default bench step with the colour or shapes streams at high priority
set -u -o pipefail
mkdir -p gpurun_out
B="python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --steps 8 --warmup 2"
for rep in 1 2; do
for env in "LLFE_NONE=0" "LLFE_COLOUR_PRIORITY=1" "LLFE_SHAPES_PRIORITY=1"; do
  for pl in on off; do
    env $env timeout -k 10 300 $B --pipeline $pl > gpurun_out/prio.json 2> gpurun_out/prio.err || { tail -3 gpurun_out/prio.err; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/prio.json').read().strip().splitlines()[-1])
print('%-24s pipeline %-3s img/s %8.0f step %6.2f' % (sys.argv[1], sys.argv[2], d['value'], d['ms_per_step']))" "$env" $pl
  done
done
done
