#!/bin/bash
# The bench lines of the four workloads with the committed r06zz counter summaries joined
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06zz_lines
mkdir -p "$OUT"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
for wl in rmat backbone arxiv; do
  timeout -k 10 400 python bench.py --workload $wl --steps 5 --warmup 2 > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "$wl rc=$?"; exit 1; }
done
for wl in roman rmat backbone arxiv; do
  python3 -c "import json;a=json.load(open('$OUT/bench_$wl.json'));r=a['roofline'];print('$wl',a['ms_per_step'],r.get('frac'),r.get('traffic'),str(r.get('basis'))[:80])"
done
