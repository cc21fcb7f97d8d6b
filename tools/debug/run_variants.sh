#!/bin/bash
# GPU box: time each tools/debug/variants/libllfe_*.so on the bench workload (stencil
# isolated time and the step); the in-tree libllfe.so is restored afterwards.
set -u -o pipefail
mkdir -p gpurun_out
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --pipeline off --steps 5 --warmup 2 "$@" \
        > gpurun_out/var.json 2> gpurun_out/var.err || { echo "$v failed"; tail -3 gpurun_out/var.err; cp /tmp/libllfe_keep.so $L; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/var.json').read().strip().splitlines()[-1])
k=d['kernels']
iso=' '.join('%s %.3f' % (n.replace('k_', ''), v.get('isolated_ms') or 0) for n, v in k.items())
pc = d.get('per_class') or {}
pcs = ' | ' + ' '.join('%s %.0f' % (c, v['value']) for c, v in pc.items()) if pc else ''
print('%-28s img/s %8.0f step %6.2f | iso: %s%s' % (sys.argv[1], d['value'], d['ms_per_step'], iso, pcs))
" "$(basename $v)"
done
cp /tmp/libllfe_keep.so $L
