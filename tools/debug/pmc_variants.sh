#!/bin/bash
# GPU box: one PMC pass (tools/pmc.sh) per tools/debug/variants/libllfe_*.so
#   tools/debug/pmc_variants.sh "COUNTERS" [kernel-regex] [summary-grep] [features]
set -u -o pipefail
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    n=$(basename $v .so)
    echo "== $n"
    bash tools/pmc.sh $n "$1" "${2:-k_kmeans}" --features "${4:-colors}" | grep -E "${3:-k_kmeans<true>}" || { cp /tmp/libllfe_keep.so $L; exit 1; }
done
cp /tmp/libllfe_keep.so $L
