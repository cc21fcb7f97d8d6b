#!/bin/bash
# GPU box (one GPU): the driver's N=2 command line with default arguments, both ranks on
# cuda:0 (LLFE_BENCH_SHARE_GPU=1) -- the default world > 1 path end to end
set -u -o pipefail
mkdir -p gpurun_out
LLFE_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29523 bench.py --gpus 2 --steps 5 --warmup 2 \
    > gpurun_out/share2_default.json 2> gpurun_out/share2_default.err || { tail -20 gpurun_out/share2_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/share2_default.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value','n_gpus','ms_per_step','host_contour_busy')}, d['config']['contours'], d['e2e_png'], (d['per_class'] or {}).keys())"
