#!/bin/bash
# GPU box: results of every tools/debug/variants/libllfe_*.so (loaded through LLFE_LIB_PATH,
# so older builds need not carry every later entry point) and of the in-tree build on one
# batch, compared with the first variant (bit identity of k-means / shapes / shadows)
set -u -o pipefail
first=""
for v in ${ID_VARIANTS:-tools/debug/variants/libllfe_k_final.so} intree; do
    if [ "$v" = intree ]; then n=intree; lp=low_level_feature_extraction_amd/libllfe.so; else n=$(basename $v .so); lp=$v; fi
    LLFE_LIB_PATH=$lp timeout -k 10 300 python3 tools/debug/dump_results.py /tmp/res_$n.npz ${ID_N:-128} 2> gpurun_out/id_$n.err || { echo "$n failed"; tail -3 gpurun_out/id_$n.err; exit 1; }
    if [ -z "$first" ]; then first=$n; continue; fi
    python3 -c "
import numpy as np, sys
a, b = np.load('/tmp/res_$first.npz'), np.load('/tmp/res_$n.npz')
bad = [k for k in a.files if k in b.files and not np.array_equal(a[k], b[k])]
print('$n vs $first:', 'IDENTICAL' if not bad else 'DIFFERENT in ' + ', '.join(bad))
"
done
