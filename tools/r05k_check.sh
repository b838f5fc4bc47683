#!/bin/bash
# Round-5: kernel trace of the R-MAT-22 Jaccard-T step (the candidate top-k's kernels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r05k}
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
f=$(find "$OUT/trace" -name "*kernel_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-8
