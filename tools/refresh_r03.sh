#!/bin/bash
# GPU box, round 3 evidence.  The GPU suite and smoke; then per workload: the
# rocprofv3 summaries first (kernel trace + FETCH / WRITE / L2 / SQ passes, the
# summary stamped with the sources' hash), installed under profiles/ as
# TAG_<key>_pmc_summary.json so that the bench line run next joins its own
# counters; then the bench line with its CPU baseline.  Then the sharded-Jaccard
# per-rank probe and the drop-in API timer.  usage: refresh_r03.sh TAG [workloads...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r03f}; shift
O=gpurun_out/$T
mkdir -p "$O"
W=${*:-suite roman rmat arxiv backbone api}
for w in $W; do
  case $w in
    suite)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
      tail -1 "$O/pytest_gpu.log"
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log"
      continue ;;
    api)
      timeout -k 10 300 python tools/api_timer.py > "$O/api_timer.json" 2> "$O/api_timer.err" || { tail -10 "$O/api_timer.err"; exit 1; }
      cat "$O/api_timer.json"
      continue ;;
    shares)
      timeout -k 10 300 python tools/shares_probe.py 22 3 > "$O/rmat_shares_probe.json" 2> "$O/rmat_shares_probe.err" || { tail -10 "$O/rmat_shares_probe.err"; exit 1; }
      cat "$O/rmat_shares_probe.json"
      continue ;;
    roman) args=""; key=roman ;;
    rmat) args="--workload rmat"; key=rmat ;;
    arxiv) args="--workload arxiv"; key=arxiv ;;
    backbone) args="--workload backbone"; key=backbone-rmat18 ;;
  esac
  bash tools/profile_bench.sh "$O/prof_$key" $args > "$O/prof_$key.log" 2>&1 || { tail -10 "$O/prof_$key.log"; exit 1; }
  tail -1 "$O/prof_$key.log"
  cp "$O/prof_$key/pmc_summary.json" "profiles/${T}_${key}_pmc_summary.json"
  extra=""; [ "$w" = backbone ] && extra="--steps 2 --warmup 1"
  timeout -k 10 600 python bench.py $args $extra > "$O/${key}_bench.json" 2> "$O/${key}_bench.err" || { tail -10 "$O/${key}_bench.err"; exit 1; }
  cat "$O/${key}_bench.json"
done
