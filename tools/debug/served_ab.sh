set -u -o pipefail
ARGS="--cpu-baseline off --e2e-host-steps 0 --e2e-png-steps 0 --e2e-jpeg-steps 0 --per-class-steps 0"
for d in 2 3; do
timeout -k 10 300 python bench.py $ARGS --batcher-inflight $d > gpurun_out/sv_$d.json 2> gpurun_out/sv_$d.err || { tail -20 gpurun_out/sv_$d.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('gpurun_out/sv_$d.json').read().strip().splitlines()[-1]); s=d['served_batcher']
print('depth $d value %.0f served %.0f ratio %.3f worker %s mean_launch %s' % (d['value'], s['value'], s['ratio_to_value'], s['worker'], s['mean_launch']))"
done
