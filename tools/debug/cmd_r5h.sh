#!/bin/bash
# GPU box (round 5): the serving-thread GC stall -- pipelined timeline with and without
# gc.freeze, then the headline (current tree, gc.freeze in bench.py) against the round-4 build.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for fz in 0 1; do
    PIPE_FREEZE=$fz timeout -k 10 300 python tools/debug/pipe_timeline.py gpurun_out/r5h_pipe_fz$fz.txt 12 2 > gpurun_out/r5h_pipe_fz$fz.log 2>&1 || { tail -20 gpurun_out/r5h_pipe_fz$fz.log; exit 1; }
    head -1 gpurun_out/r5h_pipe_fz$fz.log; grep "host collect" gpurun_out/r5h_pipe_fz$fz.txt | awk '{printf "%s:%.1f ", $3, $5-$4} END {print ""}'
done
A="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --steps 20 --warmup 5"
for i in 1 2; do
    for t in r4 cur; do
        if [ $t = r4 ]; then d=tools/debug/r4tree; else d=.; fi
        (cd $d && timeout -k 10 240 python bench.py $A) > gpurun_out/r5h_${t}_$i.json 2> gpurun_out/r5h_${t}_$i.err \
            || { echo "$t $i failed"; tail -5 gpurun_out/r5h_${t}_$i.err; exit 1; }
        python3 -c "
import json
d=json.loads(open('gpurun_out/r5h_${t}_$i.json').read().strip().splitlines()[-1])
k=d['kernels']
print('$t $i', d['value'], d['ms_per_step'], 'one-at-a-time', d.get('value_one_batch_at_a_time'), 'serving', d.get('serving_thread'), 'asm', d['result_assembly']['host_cpu_ms_per_step'], 'stencil iso', k['k_stencil'].get('isolated_ms'), 'kmeans', k['k_kmeans']['avg_ms'])"
    done
done
