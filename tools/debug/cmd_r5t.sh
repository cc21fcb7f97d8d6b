#!/bin/bash
# GPU box (round 5): per-class (ui / photo / mix) kernel times of the shapes + shadows path
# (stencil + hysteresis chain) from rocprofv3 kernel traces, for each tools/debug/variants
# build given as arguments (default: the in-tree build).  Traces stay in /tmp; only the
# summaries come back.
set -u -o pipefail
mkdir -p gpurun_out/r5t
export TMPDIR=/tmp
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in "${@:-}"; do
    [ -n "$v" ] && cp tools/debug/variants/libllfe_$v.so $L
    for k in ui photo mix; do
        D=/tmp/r5t_${v}_$k; rm -rf $D
        timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $D -o run --output-format csv -- python3 tools/debug/stencil_kind.py $k > gpurun_out/r5t/${v}_$k.log 2>&1 || { tail -5 gpurun_out/r5t/${v}_$k.log; cp /tmp/libllfe_keep.so $L; exit 1; }
        f=$(find $D -name '*kernel_stats.csv' | head -1)
        echo "== ${v:-intree} $k"
        python3 - "$f" <<'PY' | tee -a gpurun_out/r5t/summary.txt
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r['Name']
    if 'llfe' in n:
        print('%-30s %5s avg %9.1f us min %9.1f' % (n.split('(anonymous namespace)::')[-1].split('(')[0][:30], r['Calls'], float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3))
PY
    done
done
cp /tmp/libllfe_keep.so $L
