#!/bin/bash
# GPU box: kernel timelines of the pipelined headline for the round-4 build (tools/debug/r4tree)
# and the current tree, with each llfe kernel's start / end relative to its step's k_kmeans
# start (two steps), to see where the overlap of two batches in flight went.
set -u -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tl_ab
for t in r4 cur; do
    if [ $t = r4 ]; then d=tools/debug/r4tree; else d=.; fi
    rm -rf /tmp/tl_$t
    (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "llfe" -d /tmp/tl_$t -o run --output-format csv -- \
        python3 bench.py --steps 8 --warmup 2 --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 \
        --per-class-steps 0) > gpurun_out/tl_ab/${t}_bench.json 2> gpurun_out/tl_ab/${t}.err || { tail -5 gpurun_out/tl_ab/${t}.err; exit 1; }
    f=$(find /tmp/tl_$t -name '*kernel_trace.csv' | head -1)
    python3 - "$f" $t <<'PY' | tee gpurun_out/tl_ab/$t.txt
import csv, re, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'llfe::' in r['Kernel_Name']]
def short(n):
    m = re.search(r'(k_\w+)', n)
    return m.group(1) if m else n[:40]
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']), r.get('Queue_Id', r.get('Stream_Id', ''))) for r in rows)
km = [x for x in iv if x[2] == 'k_kmeans']
print(sys.argv[2], 'kernels', len(iv), 'k_kmeans launches', len(km))
for i in range(len(km) - 5, len(km) - 2):
    a, b = km[i], km[i + 1]
    print('--- step: k_kmeans %d, start-to-start %.2f ms' % (i, (b[0] - a[0]) / 1e6))
    for s, e, n, q in iv:
        if a[0] - 12e6 <= s < b[0]:
            print('  %-22s q%-3s start %+8.3f end %+8.3f ms (%.3f)' % (n, q, (s - a[0]) / 1e6, (e - a[0]) / 1e6, (e - s) / 1e6))
PY
done
