set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/identity.sh 2>&1 | grep -v "^$" || exit 1
bash tools/debug/run_variants.sh || exit 1
bash tools/debug/pipe_variants.sh || exit 1
