set -u -o pipefail
mkdir -p gpurun_out
B="python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --steps 20 --warmup 5"
for d in 2 3 2 3; do
  for cfg in "c2:--batch 256 --features colors,shapes" "c3:--batch 512"; do
    name=${cfg%%:*}; a=${cfg#*:}
    LLFE_INFLIGHT=$d timeout -k 10 300 $B $a > gpurun_out/if_${name}_$d.json 2> gpurun_out/if_${name}_$d.err || { tail -3 gpurun_out/if_${name}_$d.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/if_${name}_$d.json').read().strip().splitlines()[-1])
print('$name inflight $d: %.0f images/s, %.2f ms/step, asm %.2f ms/step' % (d['value'], d['ms_per_step'], d['result_assembly']['host_cpu_ms_per_step']))"
  done
done
