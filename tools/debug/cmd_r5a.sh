#!/bin/bash
# GPU box (round 5): k-means split variants -- bit identity vs the round-4 kernel, per-phase
# slot gaps (LLFE_KM_TRACE), isolated k_kmeans time and the step.
set -u -o pipefail
mkdir -p gpurun_out
L=low_level_feature_extraction_amd/libllfe.so
timeout -k 10 600 bash tools/debug/identity.sh || exit 1
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
# PMC calibration: what one instruction of each kind counts as in SQ_INSTS_VALU
cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d /tmp/vc -o vc --output-format csv -- $GRAFT_REPO_ROOT/tools/debug/valu_count > $GRAFT_REPO_ROOT/gpurun_out/valu_count.log 2>&1; cd $GRAFT_REPO_ROOT && find /tmp/vc -name "*counter_collection*" -exec cp {} gpurun_out/valu_count_pmc.csv \; ; true
