#!/bin/bash
# GPU box: the end-to-end lines (decoded arrays, PNG bytes, JPEG bytes) with the contour
# pass on the host pool and on the GPU (which mode the auto rule
# should pick when the host also decodes).  gpurun_out/e2e/*.json
set -u -o pipefail
O=gpurun_out/e2e
mkdir -p $O
B="python bench.py --cpu-baseline off --per-class-steps 0 --steps 3 --warmup 1 --e2e-png-steps 4 --e2e-jpeg-steps 4 --e2e-host-steps 6"
timeout -k 10 400 $B --contours host > $O/e2e_host_contours.json &&
timeout -k 10 400 $B --contours gpu > $O/e2e_gpu_contours.json
