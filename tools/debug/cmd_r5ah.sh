#!/bin/bash
# GPU box (round 5): run-based hysteresis (k_ccl_runs, block-level work counter) after the
# per-wave counter version faulted: the canny / shape-mask parity tests first, then identity
# of every variant vs round 4's kernels, isolated times, per-class traces, the GPU tests and
# the headline bench of the in-tree build.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 60 --timeout-method thread -k "canny or shape_mask or dilate" > gpurun_out/r5ah_parity.log 2>&1; rc=$?; tail -2 gpurun_out/r5ah_parity.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5ah_identity.log 2>&1; rc=$?; cat gpurun_out/r5ah_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5ah_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
rm -f gpurun_out/r5t/summary.txt
timeout -k 10 900 bash tools/debug/cmd_r5t.sh k_final q_nolist || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5ah_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5ah_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0 > gpurun_out/r5ah_bench.json 2> gpurun_out/r5ah_bench.err || { tail -5 gpurun_out/r5ah_bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r5ah_bench.json').read().strip().splitlines()[-1])
k=d['kernels']
print('img/s %.0f step %.2f one-at-a-time %.0f' % (d['value'], d['ms_per_step'], d.get('value_one_batch_at_a_time') or 0), ' '.join('%s %.3f/%.3f' % (n, v['avg_ms'], v.get('isolated_ms') or 0) for n, v in k.items()))"
