#!/bin/bash
# GPU box: SQ counters of k_stencil_stream per synthetic class (3 launches of 512 x 1080p
# each, tools/debug/stencil_kind.py), one rocprofv3 --pmc pass per class (8 SQ counters).
set -u -o pipefail
O=gpurun_out/stencil_pmc_kind
mkdir -p $O
rm -f $O/summary.txt
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
for k in photo ui mix; do
    rm -rf /tmp/spk_$k
    timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace \
        -d /tmp/spk_$k -o run --output-format csv -- python3 tools/debug/stencil_kind.py $k > $O/$k.log 2>&1 \
        || { tail -5 $O/$k.log; exit 1; }
    f=$(find /tmp/spk_$k -name '*counter_collection.csv' | head -1)
    python3 -c "
import csv, sys
r = csv.DictReader(open(sys.argv[1])); w = csv.DictWriter(open(sys.argv[2], 'w'), r.fieldnames); w.writeheader()
[w.writerow(x) for x in r if 'k_stencil_stream' in x['Kernel_Name']]" "$f" $O/$k.csv
    python3 - "$f" $k <<'PY' | tee -a $O/summary.txt
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_stencil_stream" in r["Kernel_Name"]]
agg = collections.defaultdict(float)
disp = set()
for r in rows:
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
per = {k: v / n for k, v in agg.items()}
steps = 40 * 225.0 * 512  # waves x full row steps (ya - 5 .. yb + 5, from row 0) per launch, 512 x 1080p, 216-row segments
print(sys.argv[2], "dispatches", n, {k: "%.4g" % v for k, v in sorted(per.items())},
      "VALU per wave-step %.1f" % (per.get("SQ_INSTS_VALU", 0) / steps))
PY
done
