#!/bin/bash
# Copy the summaries of one tools/refresh.sh run (gpurun_out/TAG, merged back
# from the GPU box) into profiles/ under the same tag.  usage: collect_profiles.sh TAG
set -e
cd "$(dirname "$0")/.."
TAG=$1
S=gpurun_out/$TAG
D=profiles
[ -d "$S" ] || { echo "no $S"; exit 1; }
for f in "$S"/*_bench.json; do cp "$f" "$D/${TAG}_$(basename "$f")"; done
[ -f "$S/pytest_gpu.log" ] && tail -3 "$S/pytest_gpu.log" > "$D/${TAG}_pytest_gpu_summary.txt"
for p in "$S"/prof_*; do
  [ -d "$p" ] || continue
  w=$(basename "$p"); w=${w#prof_}
  [ -f "$p/trace/run_kernel_stats.csv" ] && cp "$p/trace/run_kernel_stats.csv" "$D/${TAG}_${w}_kernel_stats.csv"
  [ -f "$p/pmc_summary.json" ] && cp "$p/pmc_summary.json" "$D/${TAG}_${w}_pmc_summary.json"
done
ls "$D" | grep "^${TAG}_"
