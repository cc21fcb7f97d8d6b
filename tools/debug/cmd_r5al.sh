#!/bin/bash
# GPU box (round 5, last): the build without the unused second tile list: identity vs round
# 4's kernels, smoke, the GPU tests, the headline bench (no side legs).
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5al_identity.log 2>&1; rc=$?; cat gpurun_out/r5al_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5al_identity.log && exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5al_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r5al_smoke.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5al_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r5al_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 > gpurun_out/r5al_bench.json 2> gpurun_out/r5al_bench.err || { tail -5 gpurun_out/r5al_bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5al_bench.json').read().strip().splitlines()[-1])
print('img/s %.0f step %.2f' % (d['value'], d['ms_per_step']), {k: (v['value'], v['ms_per_step']) for k, v in d['per_class'].items()})"
