#!/bin/bash
# GPU box (round 5): the pipelined headline, round-4 build (tools/debug/r4tree, built from
# commit d4ff106) vs the current tree, alternated on one box; then the stencil's VALU count
# per synthetic class.
set -u -o pipefail
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
A="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --steps 20 --warmup 5"
for i in 1 2 3; do
    for t in r4 cur; do
        if [ $t = r4 ]; then d=tools/debug/r4tree; else d=.; fi
        (cd $d && timeout -k 10 240 python bench.py $A) > gpurun_out/ab/${t}_$i.json 2> gpurun_out/ab/${t}_$i.err \
            || { echo "$t $i failed"; tail -5 gpurun_out/ab/${t}_$i.err; exit 1; }
        python3 -c "
import json
d=json.loads(open('gpurun_out/ab/${t}_$i.json').read().strip().splitlines()[-1])
k=d['kernels']
print('$t $i', d['value'], d['ms_per_step'], 'one-at-a-time', d.get('value_one_batch_at_a_time'), 'asm', d['result_assembly']['host_cpu_ms_per_step'], 'contour busy', d.get('host_contour_busy'), {n: (v['avg_ms'], v['isolated_ms']) for n, v in k.items()})"
    done
done
timeout -k 10 600 bash tools/debug/stencil_pmc_kind.sh || exit 1
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5e_identity.log 2>&1; echo "identity rc=$?"; cat gpurun_out/r5e_identity.log
timeout -k 10 600 bash tools/debug/run_variants.sh || exit 1
