#!/bin/bash
# GPU box: the -k selected GPU tests (default: the colour path) against every
# tools/debug/variants/libllfe_*.so; the in-tree libllfe.so is restored afterwards.
set -u -o pipefail
mkdir -p gpurun_out
K=${1:-"unique or parity or ragged or pipeline or configs"}
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep.so
for v in tools/debug/variants/libllfe_*.so; do
    cp "$v" $L
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/tv.log 2>&1
    rc=$?
    echo "$(basename $v): $(tail -1 gpurun_out/tv.log)"
    if [ $rc -ne 0 ]; then tail -30 gpurun_out/tv.log; cp /tmp/libllfe_keep.so $L; exit $rc; fi
done
cp /tmp/libllfe_keep.so $L
