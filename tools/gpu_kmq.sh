#!/bin/bash
# GPU box: k-means parity tests, then the per-attempt k-means timeline and one bench line
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_kmq_tests.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_kmq_tests.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/km_trace.sh || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 > gpurun_out/bench_kmq.json 2> gpurun_out/bench_kmq.err || exit 1
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/bench_kmq.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k: (v['avg_ms'], v.get('isolated_ms')) for k, v in d['kernels'].items()})
PY
