#!/bin/bash
# GPU box (round 6, final build): bench.py on every BASELINE config that fits one GPU, pipelined, with the CPU
# baseline of the same config from decoded arrays and from PNG bytes (one JSON line each,
# gpurun_out/configs_r6/*.json).  configs[0] (one 512x512 PNG through the CPU plumbing) gets
# its CPU rate from the same harness at 512x512 (the GPU line there is a 64-image batch of
# the drop-in path, not the reference's single-image call).
set -u -o pipefail
O=gpurun_out/configs_r6
mkdir -p $O
B="python bench.py --cpu-input both --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --batcher-steps 0 --steps 20 --warmup 5"
timeout -k 10 300 $B --batch 64 --height 512 --width 512 --features colors --cpu-images 64 > $O/c0_512_colors.json &&
timeout -k 10 400 $B --batch 256 --features colors > $O/c1_colors_256.json &&
timeout -k 10 400 $B --batch 256 --features colors,shapes > $O/c2_colors_shapes_256.json &&
timeout -k 10 400 $B --batch 512 > $O/c3_full_512.json &&
timeout -k 10 500 $B --batch 128 --height 2160 --width 3840 --preprocessing high_quality --cpu-images 16 > $O/c4_4k_full_128.json || exit 1
# the driver's N = 2 command shape, two ranks sharing this box's one GPU (LLFE_BENCH_SHARE_GPU)
LLFE_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 \
    --e2e-host-steps 0 --per-class-steps 0 --batcher-steps 0 > $O/share2_full_512.json
