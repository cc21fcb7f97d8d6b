#!/bin/bash
# GPU box: the pipelined headline (driver's 20 steps / 5 warm-up, no side legs) for each
# tools/debug/variants/libllfe_*.so, twice in alternation; the in-tree libllfe.so is restored
set -u -o pipefail
mkdir -p gpurun_out
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep_p.so
for r in 1 2; do
  for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 "$@" \
        > gpurun_out/pv.json 2> gpurun_out/pv.err || { echo "$v failed"; tail -3 gpurun_out/pv.err; cp /tmp/libllfe_keep_p.so $L; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/pv.json').read().strip().splitlines()[-1])
print('%-24s pipelined %8.0f img/s step %6.2f ms | one-at-a-time %8.0f | kmeans iso %.3f' % (sys.argv[1], d['value'], d['ms_per_step'], d.get('value_one_batch_at_a_time') or 0, d['kernels']['k_kmeans']['isolated_ms']))" "$(basename $v .so)"
  done
done
cp /tmp/libllfe_keep_p.so $L
