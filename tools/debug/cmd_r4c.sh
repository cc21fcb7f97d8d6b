set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/identity.sh || exit 1
bash tools/debug/km_trace_variants.sh 2>&1 | grep -E "^==|photo|ui |span" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_served.py -m gpu -x -q --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/tests_r4c.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r4c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 > gpurun_out/bench_r4c.json 2> gpurun_out/bench_r4c.err || { tail -5 gpurun_out/bench_r4c.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_r4c.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'one-at-a-time', d['value_one_batch_at_a_time'])
print('roof', d['roofline'])
print({k:(v['avg_ms'], v.get('isolated_ms')) for k,v in d['kernels'].items()})
"
