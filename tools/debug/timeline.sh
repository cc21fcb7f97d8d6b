#!/bin/bash
# GPU box: llfe kernel timeline of a pipelined bench run (kernel trace, llfe kernels only),
# summarised on the box: device busy fraction (union of kernel intervals) and the gaps.
set -u -o pipefail
export TMPDIR=/tmp
rm -rf /tmp/tl
timeout -k 10 300 rocprofv3 --kernel-trace --kernel-include-regex "llfe" -d /tmp/tl -o run --output-format csv -- \
    python3 bench.py --steps 6 --warmup 2 --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 \
    --per-class-steps 0 "$@" > gpurun_out/tl_bench.json 2> gpurun_out/tl.err || { tail -5 gpurun_out/tl.err; exit 1; }
python3 - <<'PY'
import csv, re
rows = [r for r in csv.DictReader(open('/tmp/tl/run_kernel_trace.csv')) if 'llfe::' in r['Kernel_Name']]
def short(n):
    m = re.search(r'(k_\w+)', n)
    return m.group(1) if m else n[:40]
iv = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name'])) for r in rows)
km = [x for x in iv if x[2] == 'k_kmeans']
print('kernels', len(iv), 'k_kmeans launches', len(km))
t0, t1 = km[2][0], km[-3][1]  # skip warm-up launches at both ends
sel = [x for x in iv if x[1] > t0 and x[0] < t1]
busy = 0; cur_s = cur_e = None; gaps = []
for s, e, n in sel:
    s, e = max(s, t0), min(e, t1)
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s; gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = t1 - t0
print('window %.2f ms, device busy (some llfe kernel running) %.1f %%, gaps %d, total gap %.3f ms' % (span / 1e6, 100 * busy / span, len(gaps), sum(g for g, _ in gaps) / 1e6))
for g, n in sorted(gaps, reverse=True)[:12]: print('  gap %.3f ms before %s' % (g / 1e6, n))
# per interval between consecutive k_kmeans starts: span and busy fraction
for a, b in zip(km, km[1:]):
    ws, we = a[0], b[0]
    segs = sorted((max(s, ws), min(e, we)) for s, e, _ in iv if e > ws and s < we)
    bz = 0; cs = ce = None
    for s, e in segs:
        if ce is None or s > ce:
            if ce is not None: bz += ce - cs
            cs, ce = s, e
        else: ce = max(ce, e)
    if ce is not None: bz += ce - cs
    print('k_kmeans start-to-start %.2f ms, busy %.1f %%, k_kmeans %.2f ms' % ((we - ws) / 1e6, 100 * bz / (we - ws), (a[1] - a[0]) / 1e6))
PY
