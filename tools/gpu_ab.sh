#!/bin/bash
# GPU box (round 6): identity vs round 5's final kernels, then the bench's headline and
# isolated kernel times with and without an env switch (A/B).  Usage:
#   tools/gpu_ab.sh TAG "ENV=0" [extra bench args]
set -u -o pipefail
TAG=$1; SW=$2; shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/${TAG}_identity.log 2>&1; rc=$?; cat gpurun_out/${TAG}_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/${TAG}_identity.log && exit 1
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --batcher-steps 0 $*"
for v in A B A B; do
    if [ $v = A ]; then E="$SW"; else E=""; fi
    env $E timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
    python3 - gpurun_out/${TAG}_$v.json "$v ${E:-default}" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("%-14s value %.0f ms/step %.2f one-at-a-time %.0f | " % (sys.argv[2], d["value"], d["ms_per_step"], d.get("value_one_batch_at_a_time") or 0)
      + " ".join("%s %.3f/%.3f" % (n.replace("k_", ""), v["avg_ms"], v.get("isolated_ms") or 0) for n, v in k.items()))
PY
done
