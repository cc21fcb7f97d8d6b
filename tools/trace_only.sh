#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary of a short bench run (no tests).
# Usage: tools/trace_only.sh TAG [bench args]
set -u -o pipefail
TAG=${1:-t}; shift || true
export TMPDIR=/tmp
P=/tmp/llfe_t_$TAG
rm -rf "$P"; mkdir -p gpurun_out/t_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- python3 bench.py --steps 2 \
    --warmup 1 --cpu-baseline off --e2e-png-steps 0 "$@" > gpurun_out/t_$TAG/bench_under_trace.json 2> gpurun_out/t_$TAG/trace.err \
    || { echo "trace failed"; tail -5 gpurun_out/t_$TAG/trace.err; exit 1; }
cp $P/run_kernel_stats.csv gpurun_out/t_$TAG/kernel_stats.csv
grep llfe $P/run_kernel_stats.csv | sed -E 's/^"[^"]*::([a-z_0-9<>A-Za-z]+)\([^"]*"/\1/' \
    | awk -F, '{printf "%-24s calls %4d avg %9.1f us\n", $1, $2, $4/1000}' | tee gpurun_out/t_$TAG/kernels.txt
