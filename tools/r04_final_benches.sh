#!/bin/bash
# Round-4 final bench lines of every workload (defaults, CPU baselines included).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04benches}
mkdir -p "$OUT"
for wl in rmat backbone arxiv scorers exact_er topology geodesic; do
  timeout -k 10 600 python bench.py --workload $wl > "$OUT/$wl.json" 2> "$OUT/$wl.err" || { echo "$wl rc=$?"; tail -5 "$OUT/$wl.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/$wl.json').read().strip().splitlines()[-1]);print('$wl',a['ms_per_step'],'ms/step', (a.get('cpu_baseline') or {}).get('value'))"
done
