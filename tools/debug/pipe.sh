set -u -o pipefail
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-host-steps 0 --steps 8 --warmup 2 --pipeline on > gpurun_out/pipe.json 2> gpurun_out/pipe.err || { tail -3 gpurun_out/pipe.err; exit 1; }
python3 -c "
import json
d=json.loads(open('gpurun_out/pipe.json').read().strip().splitlines()[-1])
print('pipelined', d['value'], 'one at a time', d['value_one_batch_at_a_time'], 'kmeans avg', d['kernels']['k_kmeans']['avg_ms'])
"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/ptr -o run --output-format csv -- python3 bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-host-steps 0 --steps 4 --warmup 1 --pipeline on > /dev/null 2> gpurun_out/ptr.err || { tail -3 gpurun_out/ptr.err; exit 1; }
cp /tmp/ptr/run_kernel_trace.csv gpurun_out/pipe_trace.csv
