#!/bin/bash
# Round-4 final: rocprofv3 kernel-trace + PMC summaries (tools/profile_bench.sh) of the
# bench workloads on the final sources, for bench.py's hash-checked roofline.
# usage: r04z_profiles.sh OUTDIR WORKLOAD...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04z}
shift
for wl in "$@"; do
  tools/profile_bench.sh "$OUT/$wl" --workload $wl || { echo "profile $wl rc=$?"; exit 1; }
  echo "$wl: $(head -c 300 $OUT/$wl/bench_trace.json)"
done
