#!/bin/bash
# GPU box: tools/debug/shadow_check.py with each tools/debug/variants/libllfe_*.so
set -u -o pipefail
mkdir -p gpurun_out
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    echo "== $v"
    timeout -k 10 300 python -u tools/debug/shadow_check.py 2>&1 | grep -v amdgpu.ids | tail -13 || { echo "$v failed"; cp /tmp/libllfe_keep.so $L; exit 1; }
done
cp /tmp/libllfe_keep.so $L
