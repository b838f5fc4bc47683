#!/bin/bash
# Round-4 l: counters of the RMAT-18 backbone prune on the current sources.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04l}
mkdir -p "$OUT"
tools/profile_bench.sh "$OUT/backbone" --workload backbone || exit $?
cat "$OUT/backbone/pmc_summary.txt" | head -40
