#!/bin/bash
# GPU box (round 5): identity of the k-means / stencil variants vs the round-4 build, the
# GPU test suite on the in-tree build, k-means slot gaps per variant, timings, and the
# SQ_INSTS_VALU calibration.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5c_identity.log 2>&1; echo "identity rc=$?" ; cat gpurun_out/r5c_identity.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/r5c_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep2.so
for v in tools/debug/variants/libllfe_*.so; do
    n=$(basename $v .so)
    cp $v $L
    rm -f gpurun_out/kt_$n.txt
    LLFE_KM_TRACE=gpurun_out/kt_$n.txt timeout -k 10 300 python bench.py --features colors --steps 1 --warmup 1 --pipeline off \
        --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 > /dev/null 2> gpurun_out/kt_$n.err \
        || { echo "$n trace failed"; tail -3 gpurun_out/kt_$n.err; cp /tmp/libllfe_keep2.so $L; exit 1; }
    echo "== $n"; python3 tools/km_trace_summary.py gpurun_out/kt_$n.txt -1
done
cp /tmp/libllfe_keep2.so $L
timeout -k 10 900 bash tools/debug/run_variants.sh || exit 1
cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d /tmp/vc -o vc --output-format csv -- $GRAFT_REPO_ROOT/tools/debug/valu_count > $GRAFT_REPO_ROOT/gpurun_out/valu_count.log 2>&1; cd $GRAFT_REPO_ROOT && find /tmp/vc -name "*counter_collection*" -exec cp {} gpurun_out/valu_count_pmc.csv \; ; true
