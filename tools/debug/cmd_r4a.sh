set -u -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 > gpurun_out/bench_asm.json 2> gpurun_out/bench_asm.err || { tail -5 gpurun_out/bench_asm.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/bench_asm.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'one-at-a-time', d['value_one_batch_at_a_time'])
print('asm', d['result_assembly'])
print('roof', d['roofline'])
print({k:(v['avg_ms'], v.get('isolated_ms')) for k,v in d['kernels'].items()})
"
bash tools/debug/km_trace_variants.sh
