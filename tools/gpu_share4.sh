#!/bin/bash
# GPU box (one GPU): rehearse the N=4 bench path -- four ranks under torch.distributed.run
# sharing cuda:0 (LLFE_BENCH_SHARE_GPU=1: gloo control plane), default 512 images per rank,
# two batches in flight, with the e2e legs (LOCAL_WORLD_SIZE=4: each rank's decode / contour
# pools get a quarter of the usable cores).  The real N>1 runs are the driver's.
set -u -o pipefail
mkdir -p gpurun_out
LLFE_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
    --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 3 --warmup 1 \
    --cpu-baseline off --e2e-png-steps 2 --e2e-jpeg-steps 2 --e2e-host-steps 2 --e2e-at-scale on --per-class-steps 0 \
    > gpurun_out/share4.json 2> gpurun_out/share4.err || { tail -20 gpurun_out/share4.err; exit 1; }
cat gpurun_out/share4.json | head -c 3000; echo
