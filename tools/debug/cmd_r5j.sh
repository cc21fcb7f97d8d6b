#!/bin/bash
# GPU box (round 5): the headline with more HIP hardware queues (GPU_MAX_HW_QUEUES 4 / 8 /
# 16, alternated), then k-means' SQ counters split by phase (the LLFE_KM_SPLIT build: one
# launch for k-means++, one for Lloyd; colours-only steps).
set -u -o pipefail
mkdir -p gpurun_out/r5j
export TMPDIR=/tmp
A="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --steps 20 --warmup 5"
for i in 1 2; do
    for q in 4 8 16; do
        GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py $A > gpurun_out/r5j/hwq${q}_$i.json 2> gpurun_out/r5j/hwq${q}_$i.err \
            || { echo "hwq $q failed"; tail -5 gpurun_out/r5j/hwq${q}_$i.err; exit 1; }
        python3 -c "
import json
d=json.loads(open('gpurun_out/r5j/hwq${q}_$i.json').read().strip().splitlines()[-1])
print('GPU_MAX_HW_QUEUES=$q run $i', d['value'], d['ms_per_step'], d.get('serving_thread'))"
    done
done
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/libllfe_keep3.so
cp tools/debug/pmcvar/libllfe_k_split.so $L
for P in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY"; do
    rm -rf /tmp/kmp
    timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d /tmp/kmp -o run --output-format csv -- python3 bench.py --features colors \
        --pipeline off --steps 2 --warmup 1 --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 \
        > gpurun_out/r5j/kmp.json 2> gpurun_out/r5j/kmp.err || { echo "pmc failed"; tail -5 gpurun_out/r5j/kmp.err; cp /tmp/libllfe_keep3.so $L; exit 1; }
    f=$(find /tmp/kmp -name '*counter_collection.csv' | head -1)
    python3 - "$f" <<'PY' | tee -a gpurun_out/r5j/kmeans_phase_pmc.txt
import csv, sys, collections, re
agg = collections.defaultdict(float); disp = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r'k_kmeans<true, (\d)', r["Kernel_Name"])
    if not m:
        continue
    ph = {"1": "kmeans++", "2": "lloyd"}[m.group(1)]
    agg[(ph, r["Counter_Name"])] += float(r["Counter_Value"])
    disp[ph].add(r["Dispatch_Id"])
for ph in ("kmeans++", "lloyd"):
    n = max(len(disp[ph]), 1)
    print(ph, "dispatches", n, {c: "%.4g" % (v / n) for (p, c), v in sorted(agg.items()) if p == ph})
PY
done
cp /tmp/libllfe_keep3.so $L
