#!/bin/bash
# GPU box (round 5): row-indexed k_bits_dilate (o) against the final build (k): dilate /
# shape-mask parity tests, identity, isolated times, per-class traces, then the default-length
# per-class lines (12 steps) of the in-tree build.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 60 --timeout-method thread -k "canny or shape_mask or dilate" > gpurun_out/r5af_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r5af_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5af_identity.log 2>&1; rc=$?; cat gpurun_out/r5af_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5af_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
rm -f gpurun_out/r5t/summary.txt
timeout -k 10 600 bash tools/debug/cmd_r5t.sh k_final o_dilate || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 > gpurun_out/r5af_bench.json 2> gpurun_out/r5af_bench.err || { tail -5 gpurun_out/r5af_bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5af_bench.json').read().strip().splitlines()[-1])
print('img/s %.0f step %.2f' % (d['value'], d['ms_per_step']), {k: (v['value'], v['ms_per_step']) for k, v in d['per_class'].items()})"
