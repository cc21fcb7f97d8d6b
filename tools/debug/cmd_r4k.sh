set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/identity.sh 2>&1 | grep -v "^$" || exit 1
bash tools/debug/km_trace_variants.sh 2>&1 | grep -E "^==|photo|ui |span" || exit 1
bash tools/debug/pipe_variants.sh || exit 1
