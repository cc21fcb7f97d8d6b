set -u -o pipefail
mkdir -p gpurun_out
bash tools/debug/identity.sh 2>&1 | grep -v "^$" || exit 1
bash tools/debug/run_variants.sh || exit 1
L=low_level_feature_extraction_amd/libllfe.so
cp $L /tmp/keep.so
cp tools/debug/variants/libllfe_${1:-g_dedup5}.so $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "unique or kmeans" tests/test_gpu_served.py -k "unique or production_keys or headline" > gpurun_out/dedup_tests.log 2>&1; rc=$?
cp /tmp/keep.so $L
tail -3 gpurun_out/dedup_tests.log
exit $rc
