set -o pipefail
for v in km256 km256w5 km512; do
  LLFE_LIB_VARIANT=$v timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench_$v.json 2>gpurun_out/bench_$v.err || exit 1
done
timeout -k 10 300 python bench.py --cpu-baseline off > gpurun_out/bench_d.json 2>gpurun_out/bench_d.err
