#!/bin/bash
# GPU box: results of every tools/debug/variants/libllfe_*.so on one batch, compared with
# the first variant (bit identity of k-means / shapes / shadows across builds)
set -u -o pipefail
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
first=""
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    n=$(basename $v .so)
    timeout -k 10 300 python3 tools/debug/dump_results.py /tmp/res_$n.npz 128 2> gpurun_out/id_$n.err || { echo "$n failed"; tail -3 gpurun_out/id_$n.err; cp /tmp/libllfe_keep.so $L; exit 1; }
    if [ -z "$first" ]; then first=$n; continue; fi
    python3 -c "
import numpy as np, sys
a, b = np.load('/tmp/res_$first.npz'), np.load('/tmp/res_$n.npz')
bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
print('$n vs $first:', 'IDENTICAL' if not bad else 'DIFFERENT in ' + ', '.join(bad))
"
done
cp /tmp/libllfe_keep.so $L
