#!/bin/bash
# GPU box: one rocprofv3 PMC pass over a standalone binary, summarised per kernel.
#   tools/debug/pmc_bin.sh TAG "COUNTERS" binary [args...]
set -u -o pipefail
TAG=$1; COUNTERS=$2; shift 2
export TMPDIR=/tmp
P=/tmp/llfe_pmcb_$TAG
OUT=gpurun_out/pmcb_$TAG
rm -rf "$P"; mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --kernel-trace -d $P -o run --output-format csv -- "$@" \
    > "$OUT/out.txt" 2> "$OUT/err.txt" || { echo "pmc pass failed"; tail -5 "$OUT/err.txt"; exit 1; }
python3 - "$P/run_counter_collection.csv" > "$OUT/summary.txt" <<'PY'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1][:40]
    tot[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:40s} {c:28s} {v / len(disp[k]):18.1f}")
PY
cat "$OUT/summary.txt"
