#!/bin/bash
# GPU box (one GPU): rehearse the N=2 bench path -- two ranks under torch.distributed.run
# sharing cuda:0 (LLFE_BENCH_SHARE_GPU=1: gloo control plane), then the N=1 line for
# comparison.  The real N>1 runs (one rank per GPU over RCCL) are the driver's.
set -u -o pipefail
mkdir -p gpurun_out
LLFE_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --batch 256 \
    --cpu-baseline off > gpurun_out/share2.json 2> gpurun_out/share2.err || { tail -20 gpurun_out/share2.err; exit 1; }
cat gpurun_out/share2.json | head -c 1200; echo
