#!/bin/bash
# Build libllfe.so with extra flags and keep it as tools/debug/variants/libllfe_NAME.so
#   tools/debug/build_variant.sh NAME "-DFOO=1 ..."
set -eu
NAME=$1; FLAGS=${2:-}
LLFE_EXTRA_FLAGS="$FLAGS" python3 -c "import sys; sys.path.insert(0, '.'); from low_level_feature_extraction_amd import _build; _build.build(force=True)"
mkdir -p tools/debug/variants
cp low_level_feature_extraction_amd/libllfe.so tools/debug/variants/libllfe_$NAME.so
