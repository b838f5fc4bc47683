#!/bin/bash
# A/B: RMAT-22 Jaccard with the default 4 hardware queues per process vs 8
# (the Jaccard row classes run on 4 side streams beside the context stream).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04hwq}
mkdir -p "$OUT"
for q in 4 8 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/q$q.json" 2> "$OUT/q$q.err" || { echo "q$q rc=$?"; tail -5 "$OUT/q$q.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/q$q.json').read().strip().splitlines()[-1]);print('GPU_MAX_HW_QUEUES=$q',a['ms_per_step'],'ms/step')"
done
