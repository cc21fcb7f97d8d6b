#!/bin/bash
# GPU box (round 6): identity vs round 5's final kernels, the GPU test suite, smoke, the
# default bench line (TAG = $1; STEPS_ONLY=1 skips the test suite)
set -u -o pipefail
TAG=${1:-r6}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/${TAG}_identity.log 2>&1; rc=$?; cat gpurun_out/${TAG}_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/${TAG}_identity.log && exit 1
if [ "${STEPS_ONLY:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
    rc=$?; tail -6 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
    timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels"]
print("value %.0f ms/step %.2f one-at-a-time %s" % (d["value"], d["ms_per_step"], d.get("value_one_batch_at_a_time")))
print("roofline", json.dumps(d["roofline"]))
print("stencil", json.dumps(d["roofline_stencil"]))
print("served_batcher", json.dumps(d.get("served_batcher")))
for n, v in k.items():
    print("  %-22s avg %.3f iso %s" % (n, v["avg_ms"], v.get("isolated_ms")))
for e in ("e2e_host", "e2e_png", "e2e_jpeg"):
    if d.get(e): print(e, d[e]["value"])
PY
if [ "${PROFILE:-0}" = 1 ]; then
    timeout -k 10 1200 bash tools/profile.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1 || { tail -20 gpurun_out/${TAG}_profile.log; exit 1; }
    tail -45 gpurun_out/${TAG}_profile.log
fi
