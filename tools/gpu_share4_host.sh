#!/bin/bash
# GPU box: the 4-rank rehearsal (tools/gpu_share4.sh) with the contour mode forced to host
# (4 usable cores per rank): does the host pool keep up at a quarter of the cores?
set -u -o pipefail
mkdir -p gpurun_out
LLFE_CONTOURS=host LLFE_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 4 --steps 3 --warmup 1 \
    --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 \
    > gpurun_out/share4_host.json 2> gpurun_out/share4_host.err || { tail -20 gpurun_out/share4_host.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/share4_host.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['contours'], d.get('host_contour_busy'))"
