#!/bin/bash
# GPU box: tools/km_trace.sh summary per tools/debug/variants/libllfe_*.so
set -u -o pipefail
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    echo "== $(basename $v .so)"
    bash tools/km_trace.sh | tail -25 || { cp /tmp/libllfe_keep.so $L; exit 1; }
done
cp /tmp/libllfe_keep.so $L
