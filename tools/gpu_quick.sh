#!/bin/bash
# GPU box: selected GPU tests (-k expression in $1), then a bench line with extra args
set -u -o pipefail
mkdir -p gpurun_out
K=${1:-""}; shift || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > gpurun_out/gpu_quick.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_quick.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 "$@" > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
brc=$?
python3 - <<'PY'
import json
try:
    d = json.loads(open("gpurun_out/bench_quick.json").read().strip().splitlines()[-1])
except Exception as e:
    print("no bench json", e); raise SystemExit(0)
print("value", d["value"], "ms/step", d["ms_per_step"])
for k, v in d["kernels"].items():
    print(f'{k:22s} avg {v["avg_ms"]:8.3f} iso {v.get("isolated_ms")}')
print("stencil roofline", d.get("roofline_stencil"))
PY
tail -3 gpurun_out/bench_quick.err
exit $brc
