#!/bin/bash
# GPU box (round 6): the served_batcher leg beside `value` with the cgroup's CPU throttling
# (cpu.stat nr_throttled / throttled_usec deltas over the bench) for each host-thread budget
# given as an argument (LLFE_HOST_THREADS; "default" = the placement's budget).
set -u -o pipefail
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0"
st() { cat /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' '; }
for t in "$@"; do
    if [ "$t" = default ]; then unset LLFE_HOST_THREADS; else export LLFE_HOST_THREADS=$t; fi
    a=$(st)
    timeout -k 10 300 python bench.py $ARGS > gpurun_out/sc_$t.json 2> gpurun_out/sc_$t.err || { tail -20 gpurun_out/sc_$t.err; exit 1; }
    b=$(st)
    python3 - gpurun_out/sc_$t.json "$t" "$a" "$b" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s = d["served_batcher"]
def kv(x):
    it = x.split(); return {it[i]: int(it[i + 1]) for i in range(0, len(it) - 1, 2)}
a, b = kv(sys.argv[3]), kv(sys.argv[4])
dl = {k: b[k] - a[k] for k in b if k in a and k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")}
print("threads %s value %.0f served %.0f ratio %.3f worker %s host_contour_busy %s cpu.stat delta %s"
      % (sys.argv[2], d["value"], s["value"], s["ratio_to_value"], s["worker"], d.get("host_contour_busy"), dl))
PY
done
cat /sys/fs/cgroup/cpu.max 2>/dev/null
