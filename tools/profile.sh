#!/bin/bash
# GPU box: rocprofv3 kernel-trace summary + two PMC passes (FETCH_SIZE, WRITE_SIZE) of
# the bench command, then the per-launch traffic table.  Usage: tools/profile.sh TAG
# Small outputs land in gpurun_out/prof_TAG/ (copied into profiles/ afterwards).
set -u -o pipefail
TAG=${1:-run}
ROOT=$(pwd)
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
P=/tmp/llfe_prof_$TAG
rm -rf "$P"
BENCH="bench.py --steps 3 --warmup 1 --cpu-baseline off --e2e-png-steps 0 --e2e-jpeg-steps 0 --e2e-host-steps 0 --per-class-steps 0 --pipeline off"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $BENCH \
    > "$OUT/bench_under_trace.json" 2> "$OUT/trace.err" || { echo "trace pass failed"; tail -5 "$OUT/trace.err"; exit 1; }
cp $P/trace/run_kernel_stats.csv "$OUT/kernel_stats.csv"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o run --output-format csv -- python3 $BENCH \
    > "$OUT/bench_under_fetch.json" 2> "$OUT/fetch.err" || { echo "fetch pass failed"; tail -5 "$OUT/fetch.err"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o run --output-format csv -- python3 $BENCH \
    > "$OUT/bench_under_write.json" 2> "$OUT/write.err" || { echo "write pass failed"; tail -5 "$OUT/write.err"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VALU --kernel-trace -d $P/valu -o run --output-format csv -- python3 $BENCH \
    > "$OUT/bench_under_valu.json" 2> "$OUT/valu.err" || { echo "valu pass failed"; tail -5 "$OUT/valu.err"; exit 1; }
python3 tools/pmc_traffic.py $P/fetch $P/write $P/valu > "$OUT/traffic.json"
head -c 300 $P/fetch/run_counter_collection.csv > "$OUT/counter_header.txt"
cat "$OUT/kernel_stats.csv"
cat "$OUT/traffic.json"
