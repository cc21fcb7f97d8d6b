#!/bin/bash
# GPU box: parity tests + one bench line (tools/gpu_check.sh), then a rocprofv3
# kernel-trace summary of a short bench run.  Usage: tools/quick_prof.sh TAG [bench args]
set -u -o pipefail
TAG=${1:-q}; shift || true
bash tools/gpu_check.sh --cpu-baseline off "$@" || exit $?
export TMPDIR=/tmp
P=/tmp/llfe_q_$TAG
rm -rf "$P"; mkdir -p gpurun_out/q_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P -o run --output-format csv -- python3 bench.py --steps 3 \
    --warmup 1 --cpu-baseline off "$@" > gpurun_out/q_$TAG/bench_under_trace.json 2> gpurun_out/q_$TAG/trace.err \
    || { echo "trace failed"; tail -5 gpurun_out/q_$TAG/trace.err; exit 1; }
grep llfe $P/run_kernel_stats.csv | sed -E 's/^"llfe::\(anonymous namespace\)::([a-z_0-9]+)\([^"]*"/\1/' \
    | awk -F, '{printf "%-20s calls %4d avg %9.1f us\n", $1, $2, $4/1000}' | tee gpurun_out/q_$TAG/kernels.txt
