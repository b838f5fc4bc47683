#!/bin/bash
# Round-5 final B: the secondary bench lines with their CPU baselines (joined to the
# committed PMC summaries of final A), the drop-in API timers, the backbone stage probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05finalB}
mkdir -p "$OUT"
for wl in rmat backbone arxiv scorers; do
  timeout -k 10 600 python bench.py --workload $wl > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "$wl rc=$?"; tail -5 "$OUT/bench_$wl.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]);print('$wl',a['ms_per_step'],'ms/step', (a.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 300 python tools/api_timer.py > "$OUT/api_roman.json" 2> "$OUT/api_roman.err" || exit $?
timeout -k 10 300 python tools/api_timer.py rmat > "$OUT/api_rmat.json" 2> "$OUT/api_rmat.err" || exit $?
timeout -k 10 900 python -u tools/bb_stage_probe.py 18 "0.6,0.85;0.8;0.7,0.9;" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
