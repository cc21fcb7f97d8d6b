set -u -o pipefail
for f in colors,shapes,shadows colors,shapes colors,shadows; do
timeout -k 10 300 python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-host-steps 0 --steps 5 --warmup 2 --features $f > gpurun_out/f.json 2> gpurun_out/f.err || { tail -3 gpurun_out/f.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/f.json').read().strip().splitlines()[-1])
k=d['kernels']
print('%-24s img/s %8.0f step %6.2f stencil iso %.3f' % (sys.argv[1], d['value'], d['ms_per_step'], k['k_stencil']['isolated_ms']))
" $f
done
