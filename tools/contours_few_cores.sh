#!/bin/bash
# GPU box: resident headline step with the host contour pool cut to 2 threads vs the GPU
# contour path -- where §8f row 2 (GPU contours) is the faster mode.
set -u -o pipefail
mkdir -p gpurun_out
B="python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --steps 5 --warmup 2"
for t in 2 3 4; do
  LLFE_HOST_THREADS=$t LLFE_CONTOURS=host timeout -k 10 300 $B > gpurun_out/fc_host$t.json 2>/dev/null || exit 1
done
LLFE_CONTOURS=gpu timeout -k 10 300 $B > gpurun_out/fc_gpu.json 2>/dev/null || exit 1
for f in gpurun_out/fc_host2.json gpurun_out/fc_host3.json gpurun_out/fc_host4.json gpurun_out/fc_gpu.json; do
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['config']['contours'], d.get('host_contour_busy'))"
done
