#!/bin/bash
# Round-6 final, part 2: rocprofv3 summaries of the four workloads and their bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r06z}
mkdir -p "$OUT"
for wl in roman rmat backbone arxiv; do
  tools/profile_bench.sh "$OUT/prof_$wl" --workload $wl || { echo "profile $wl rc=$?"; exit 1; }
  echo "$wl profiled"
done
for wl in rmat backbone arxiv; do
  timeout -k 10 400 python bench.py --workload $wl --steps 5 --warmup 2 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { tail -5 "$OUT/bench_$wl.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/bench_$wl.json'));print('$wl ms/step',a['ms_per_step'],'roofline',a['roofline'].get('frac'))"
done
