#!/bin/bash
# GPU box (round 6): SQ counters of the stencil on the 512 x 1080p mix (3 launches,
# tools/debug/stencil_kind.py), static grid (LLFE_ST_QUEUE=0) vs work queue, one
# rocprofv3 --pmc pass each (8 SQ + 1 GRBM counters), plus a kernel-trace pass for the
# durations.  Summary: gpurun_out/stencil_pmc_ab/summary.txt (round 6's is kept in
# profiles/r6/stencil_breakdown/).  The work-queue kernel was measured and removed
# (DESIGN.md §3), so both passes now run the static grid.
set -u -o pipefail
O=gpurun_out/stencil_pmc_ab
mkdir -p $O
rm -f $O/summary.txt
export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
for q in 0 1; do
    rm -rf /tmp/spq_$q /tmp/spt_$q
    LLFE_ST_QUEUE=$q timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace \
        -d /tmp/spq_$q -o run --output-format csv -- python3 tools/debug/stencil_kind.py mix > $O/q$q.log 2>&1 \
        || { tail -5 $O/q$q.log; exit 1; }
    LLFE_ST_QUEUE=$q timeout -s KILL 180 rocprofv3 --kernel-trace --stats \
        -d /tmp/spt_$q -o run --output-format csv -- python3 tools/debug/stencil_kind.py mix > $O/t$q.log 2>&1 \
        || { tail -5 $O/t$q.log; exit 1; }
    f=$(find /tmp/spq_$q -name '*counter_collection.csv' | head -1)
    t=$(find /tmp/spt_$q -name '*kernel_stats.csv' | head -1)
    python3 - "$f" "$t" $q <<'PY' | tee -a $O/summary.txt
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_stencil_stream" in r["Kernel_Name"]]
agg = collections.defaultdict(float)
disp = set()
for r in rows:
    agg[r["Counter_Name"]] += float(r["Counter_Value"])
    disp.add(r["Dispatch_Id"])
n = max(len(disp), 1)
per = {k: v / n for k, v in agg.items()}
dur = [float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(sys.argv[2])) if "k_stencil_stream" in r["Name"]]
ms = dur[0] if dur else float("nan")
slots = 1024 * 4  # SIMDs x waves per SIMD (128 VGPRs)
quads = ms * 1e-3 * 2.2e9 / 4  # quad-cycles of the launch at ~2.2 GHz
occ = per.get("SQ_WAVE_CYCLES", 0) / (slots * quads) if quads == quads else float("nan")
print("queue=%s dispatches %d ms %.3f  %s  slot-occupancy %.3f  valu-busy %.3f  active/wait/waitinst per wave-cycle %.3f/%.3f/%.3f"
      % (sys.argv[3], n, ms, {k: "%.4g" % v for k, v in sorted(per.items())}, occ,
         per.get("SQ_ACTIVE_INST_VALU", 0) / (1024 * quads),
         per.get("SQ_ACTIVE_INST_ANY", 0) / max(per.get("SQ_WAVE_CYCLES", 1), 1),
         per.get("SQ_WAIT_ANY", 0) / max(per.get("SQ_WAVE_CYCLES", 1), 1),
         per.get("SQ_WAIT_INST_ANY", 0) / max(per.get("SQ_WAVE_CYCLES", 1), 1)))
PY
done
