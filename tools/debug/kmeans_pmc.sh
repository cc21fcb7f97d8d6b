#!/bin/bash
# GPU box (round 6): SQ counters of k_kmeans (or the kernel named by $1, e.g. k_uq_part) in the bench's colour pass (one pass of 8 SQ + 1
# GRBM counters with --kernel-trace): wave-time split (issuing / parked in s_waitcnt / ready but
# not issued), VALU / SALU / LDS instruction counts per launch.
set -u -o pipefail
K=${1:-k_kmeans<}
O=gpurun_out/kmeans_pmc
[ "$K" != "k_kmeans<" ] && O=gpurun_out/pmc_$(echo $K | tr -cd 'a-z_')
mkdir -p $O
export TMPDIR=/tmp
rm -rf /tmp/kmpmc
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d /tmp/kmpmc -o run --output-format csv -- \
    python3 bench.py --features colors --steps 2 --warmup 1 --pipeline off --cpu-baseline off --e2e-host-steps 0 \
    --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --batcher-steps 0 > $O/bench.json 2> $O/pmc.err \
    || { tail -5 $O/pmc.err; exit 1; }
f=$(find /tmp/kmpmc -name '*counter_collection.csv' | head -1)
python3 - "$f" "$K" <<'PY' | tee $O/summary.txt
import csv, sys, collections
agg = collections.defaultdict(float); disp = set(); dur = {}
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] not in r["Kernel_Name"]:
        continue
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
per = {k: v / n for k, v in agg.items()}
wc = max(per.get("SQ_WAVE_CYCLES", 1), 1)
print("%s dispatches %d per launch: %s" % (sys.argv[2], n, {k: "%.4g" % v for k, v in sorted(per.items())}))
print("per wave-cycle: issuing %.3f, parked in s_waitcnt %.3f, ready not issued %.3f; VALU %.3g SALU %.3g LDS %.3g instructions"
      % (per.get("SQ_ACTIVE_INST_ANY", 0) / wc, per.get("SQ_WAIT_ANY", 0) / wc, per.get("SQ_WAIT_INST_ANY", 0) / wc,
         per.get("SQ_INSTS_VALU", 0), per.get("SQ_INSTS_SALU", 0), per.get("SQ_INSTS_LDS", 0)))
PY
