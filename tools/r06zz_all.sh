#!/bin/bash
# Round-6 final on the final sources: suite + smoke + the default line, then the
# rocprofv3 summaries of the four workloads (separate counter passes) and their lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/r06z_final.sh gpurun_out/r06zz || exit 1
for wl in roman rmat backbone arxiv; do
  tools/profile_bench.sh "gpurun_out/r06zz/prof_$wl" --workload $wl || { echo "profile $wl rc=$?"; exit 1; }
  echo "$wl profiled"
done
