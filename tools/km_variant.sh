#!/bin/bash
# GPU box: rebuild libllfe with extra compile flags (experiments), then the k-means
# timeline and one colours-only bench line.  Usage: tools/km_variant.sh "-DFOO=1" [...]
set -u -o pipefail
mkdir -p gpurun_out
for flags in "$@"; do
  LLFE_EXTRA_FLAGS="$flags" timeout -k 10 300 python -c "from low_level_feature_extraction_amd import _build; _build.build(force=True)" > gpurun_out/km_variant_build.log 2>&1 || { tail -20 gpurun_out/km_variant_build.log; exit 1; }
  echo "=== flags: $flags"
  bash tools/km_trace.sh || exit 1
done
