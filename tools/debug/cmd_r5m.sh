#!/bin/bash
# GPU box (round 5): the two halves of the Lloyd change separately (o: scalar-addressed ring
# pushes; p: per-owner LDS thresholds), identity + colours-only timing twice + VALU / SALU.
set -u -o pipefail
mkdir -p gpurun_out/r5m
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5m/identity.log 2>&1; echo "identity rc=$?"; cat gpurun_out/r5m/identity.log
timeout -k 10 600 bash tools/debug/run_variants.sh --features colors || exit 1
timeout -k 10 600 bash tools/debug/run_variants.sh --features colors || exit 1
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep5.so
for v in tools/debug/variants/libllfe_*.so; do
    cp $v $L
    rm -rf /tmp/kmv
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES --kernel-trace -d /tmp/kmv -o run --output-format csv -- python3 bench.py --features colors \
        --pipeline off --steps 2 --warmup 1 --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 \
        > gpurun_out/r5m/kmv.json 2> gpurun_out/r5m/kmv.err || { echo "pmc failed"; tail -5 gpurun_out/r5m/kmv.err; cp /tmp/libllfe_keep5.so $L; exit 1; }
    f=$(find /tmp/kmv -name '*counter_collection.csv' | head -1)
    python3 - "$f" $(basename $v) <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float); disp = set()
for r in csv.DictReader(open(sys.argv[1])):
    if "k_kmeans<" not in r["Kernel_Name"]:
        continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
print(sys.argv[2], "k_kmeans per launch", {c: "%.4g" % (v / n) for c, v in sorted(agg.items())})
PY
done
cp /tmp/libllfe_keep5.so $L
