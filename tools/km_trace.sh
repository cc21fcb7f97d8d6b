#!/bin/bash
# GPU box: k-means per-attempt timeline of one 512-image colour pass
set -u -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/km_trace.txt
LLFE_KM_TRACE=gpurun_out/km_trace.txt timeout -k 10 300 python bench.py --features colors --steps 1 --warmup 1 \
    --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 > gpurun_out/km_trace_bench.json 2> gpurun_out/km_trace.err || exit 1
python3 tools/km_trace_summary.py gpurun_out/km_trace.txt -1
