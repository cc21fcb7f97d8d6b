#!/bin/bash
# GPU box: one rocprofv3 PMC pass (counters given as one space-separated string) over a
# short colours-only (or full) bench run, summarised per kernel.
#   tools/pmc.sh TAG "SQ_WAVES SQ_WAVE_CYCLES ..." [kernel-regex] [bench args...]
set -u -o pipefail
TAG=$1; COUNTERS=$2; REGEX=${3:-llfe}; shift 3 || shift $#
export TMPDIR=/tmp
P=/tmp/llfe_pmc_$TAG
OUT=gpurun_out/pmc_$TAG
rm -rf "$P"; mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --pmc $COUNTERS --kernel-trace --kernel-include-regex "$REGEX" -d $P -o run \
    --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off --per-class-steps 0 --pipeline off "$@" \
    > "$OUT/bench.json" 2> "$OUT/err.txt" || { echo "pmc pass failed"; tail -5 "$OUT/err.txt"; exit 1; }
python3 - "$P/run_counter_collection.csv" > "$OUT/summary.txt" <<'EOF'
import csv, sys
from collections import defaultdict
tot = defaultdict(float); disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("::")[-1]
    tot[(k, r["Counter_Name"])] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
for (k, c), v in sorted(tot.items()):
    print(f"{k:28s} {c:28s} {v / len(disp[k]):18.1f}")
EOF
cat "$OUT/summary.txt"
