#!/bin/bash
# GPU box: k-means checks (incremental vs full sweeps, oracle parity, pipeline), the
# per-attempt k-means timeline, then one bench line without the CPU baseline
set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kmeans_inc.py tests/test_gpu_parity.py tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_km_tests.log 2>&1
rc=$?
tail -12 gpurun_out/gpu_km_tests.log
if [ $rc -ne 0 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
bash tools/km_trace.sh || exit 1
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench_km.json 2> gpurun_out/bench_km.err || exit 1
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/bench_km.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], {k: (v['avg_ms'], v.get('isolated_ms')) for k, v in d['kernels'].items()})
PY
