#!/bin/bash
# GPU box (round 5): GPU tests with the tile-flag hysteresis build, then the headline bench
# (pipelined, no side legs) twice.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5x_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5x_tests.log; [ $rc -eq 0 ] || exit 1
for i in 1 2; do
    timeout -k 10 300 python bench.py --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 > gpurun_out/r5x_bench$i.json 2> gpurun_out/r5x_bench$i.err || { tail -5 gpurun_out/r5x_bench$i.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/r5x_bench$i.json').read().strip().splitlines()[-1])
k=d['kernels']
print('img/s %.0f step %.2f one-at-a-time %.0f' % (d['value'], d['ms_per_step'], d.get('value_one_batch_at_a_time') or 0), ' '.join('%s %.3f/%.3f' % (n, v['avg_ms'], v.get('isolated_ms') or 0) for n, v in k.items()))"
done
