#!/bin/bash
# GPU box (round 5): where the pipelined overlap went (timelines, round-4 build vs current),
# the stencil's VALU count per synthetic class, identity + timing of the k-means variants,
# and the default bench line (serving-thread split).
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 bash tools/debug/timeline_ab.sh > gpurun_out/r5f_tl.log 2>&1 || { echo "timeline failed"; tail -20 gpurun_out/r5f_tl.log; exit 1; }
echo "timeline done"
timeout -k 10 400 bash tools/debug/stencil_pmc_kind.sh > gpurun_out/r5f_spk.log 2>&1 || { echo "stencil pmc failed"; tail -20 gpurun_out/r5f_spk.log; exit 1; }
cat gpurun_out/stencil_pmc_kind/summary.txt
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5f_identity.log 2>&1; echo "identity rc=$?"; cat gpurun_out/r5f_identity.log
timeout -k 10 600 bash tools/debug/run_variants.sh || exit 1
echo "pipelined:"; timeout -k 10 600 bash tools/debug/run_variants.sh --pipeline on --steps 12 --warmup 3 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { tail -20 gpurun_out/r5f_bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5f_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d.get('value_one_batch_at_a_time'), d.get('serving_thread'), d['result_assembly'])
for k in ('e2e_png','e2e_jpeg','e2e_jpeg_other_contour_mode'):
    v=d.get(k) or {}
    print(k, v.get('value'), v.get('decode_only'), v.get('bound'))
"
