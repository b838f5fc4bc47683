#!/bin/bash
# GPU box, round 3 evidence: every bench workload's line (with its CPU baseline)
# and its rocprofv3 summaries (kernel trace + FETCH / WRITE / L2 / SQ passes, the
# summary stamped with the sources' hash), the sharded-Jaccard per-rank probe,
# and the drop-in API timer.  usage: refresh_r03.sh TAG [workloads...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r03c}; shift
O=gpurun_out/$T
mkdir -p "$O"
W=${*:-roman rmat arxiv backbone}
for w in $W; do
  case $w in
    roman) args="" ;;
    rmat) args="--workload rmat" ;;
    arxiv) args="--workload arxiv" ;;
    backbone) args="--workload backbone --steps 2 --warmup 1" ;;
  esac
  timeout -k 10 600 python bench.py $args > "$O/${w}_bench.json" 2> "$O/${w}_bench.err" || { tail -10 "$O/${w}_bench.err"; exit 1; }
  cat "$O/${w}_bench.json"
  key=$w; [ "$w" = backbone ] && key=backbone-rmat18
  bash tools/profile_bench.sh "$O/prof_$key" $args > "$O/prof_$key.log" 2>&1 || { tail -10 "$O/prof_$key.log"; exit 1; }
  tail -1 "$O/prof_$key.log"
done
if echo "$W" | grep -q rmat; then
  timeout -k 10 300 python tools/shares_probe.py 22 3 > "$O/rmat_shares_probe.json" 2> "$O/rmat_shares_probe.err" || { tail -10 "$O/rmat_shares_probe.err"; exit 1; }
  cat "$O/rmat_shares_probe.json"
fi
timeout -k 10 300 python tools/api_timer.py > "$O/api_timer.json" 2> "$O/api_timer.err" || { tail -10 "$O/api_timer.err"; exit 1; }
cat "$O/api_timer.json"
