#!/bin/bash
# GPU box (round 5): k_uq_part marking its bitmap with a neighbour-lane dedupe and an
# unconditional OR (m) against the read-test-first form (n): identity, isolated times twice.
set -u -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 bash tools/debug/identity.sh > gpurun_out/r5ae_identity.log 2>&1; rc=$?; cat gpurun_out/r5ae_identity.log; [ $rc -eq 0 ] || exit 1
grep -q DIFFERENT gpurun_out/r5ae_identity.log && exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh || exit 1
timeout -k 10 700 bash tools/debug/run_variants.sh
