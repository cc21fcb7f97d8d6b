set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/identity.sh || exit 1
bash tools/debug/km_trace_variants.sh 2>&1 | grep -E "^==|photo|ui |span" || exit 1
bash tools/debug/run_variants.sh || exit 1
