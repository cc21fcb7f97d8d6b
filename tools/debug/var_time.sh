#!/bin/bash
# GPU box (round 6): the bench's kernel times (pipelined avg / isolated) and headline for
# each tools/debug/variants build named in the arguments, loaded through LLFE_LIB_PATH
# (timing-only builds may give wrong results), twice each, interleaved.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 --batcher-steps 0 ${VT_ARGS:-}"
for rep in 1 2; do
for v in "$@"; do
    LLFE_LIB_PATH=tools/debug/variants/libllfe_$v.so timeout -k 10 300 python bench.py $ARGS > gpurun_out/vt_$v.json 2> gpurun_out/vt_$v.err || { tail -20 gpurun_out/vt_$v.err; exit 1; }
    python3 - gpurun_out/vt_$v.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("%-14s value %.0f ms/step %.2f | " % (sys.argv[2], d["value"], d["ms_per_step"])
      + " ".join("%s %.3f/%.3f" % (n.replace("k_", ""), v["avg_ms"], v.get("isolated_ms") or 0) for n, v in k.items()))
PY
done
done
