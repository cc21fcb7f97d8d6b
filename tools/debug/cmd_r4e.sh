set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/run_variants.sh || exit 1
