#!/bin/bash
# GPU box (round 5): tools/gpu_r5.sh (tests, default bench, profile) then the in-flight depth
# comparison on BASELINE configs[2] (256 x 1080p, colors + shapes).
set -u -o pipefail
TAG=${1:-r5}
bash tools/gpu_r5.sh $TAG || exit 1
STEPS=10 bash tools/inflight_depth.sh c2 --batch 256 --features colors,shapes || exit 1
