#!/bin/bash
# GPU box: bench.py on every BASELINE config that fits one GPU (one JSON line each,
# gpurun_out/configs/*.json).  configs[0] (one PNG through the CPU plumbing) is covered
# by the drop-in tests.
set -u -o pipefail
mkdir -p gpurun_out/configs
B="python bench.py --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --steps 4 --warmup 2"
timeout -k 10 300 $B --batch 256 --features colors > gpurun_out/configs/c1_colors_256.json &&
timeout -k 10 300 $B --batch 256 --features colors,shapes > gpurun_out/configs/c2_colors_shapes_256.json &&
timeout -k 10 300 $B --batch 512 > gpurun_out/configs/c3_full_512.json &&
timeout -k 10 300 $B --batch 128 --height 2160 --width 3840 --preprocessing high_quality > gpurun_out/configs/c4_4k_full_128.json &&
timeout -k 10 300 $B --batch 512 --contours gpu > gpurun_out/configs/c3_full_512_gpu_contours.json &&
timeout -k 10 300 $B --batch 128 --height 2160 --width 3840 --preprocessing high_quality --contours gpu > gpurun_out/configs/c4_4k_full_128_gpu_contours.json
