#!/bin/bash
# GPU box, round-end refresh: full parity suite, smoke, the default bench line
# (with the CPU baseline), secondary workloads, and the rocprofv3 summaries of
# the default line.  usage: refresh.sh TAG   (e.g. r01m)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rXX}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > "$O/roman_bench.json" 2> "$O/roman_bench.err" || { tail -5 "$O/roman_bench.err"; exit 1; }
cat "$O/roman_bench.json"
timeout -k 10 300 python bench.py --workload geodesic --steps 3 --warmup 1 > "$O/geodesic_bench.json" 2> "$O/geodesic_bench.err" || { tail -5 "$O/geodesic_bench.err"; exit 1; }
cat "$O/geodesic_bench.json"
bash tools/profile_bench.sh "$O/prof_roman" > "$O/prof_roman.log" 2>&1 || { tail -5 "$O/prof_roman.log"; exit 1; }
tail -1 "$O/prof_roman.log"
if [ -n "${WITH_BACKBONE:-}" ]; then
  timeout -k 10 300 python bench.py --workload backbone --steps 1 --warmup 1 > "$O/backbone_rmat18_bench.json" 2> "$O/backbone_rmat18_bench.err" || { tail -5 "$O/backbone_rmat18_bench.err"; exit 1; }
  cat "$O/backbone_rmat18_bench.json"
  bash tools/profile_bench.sh "$O/prof_backbone-rmat18" --workload backbone > "$O/prof_backbone.log" 2>&1 || { tail -5 "$O/prof_backbone.log"; exit 1; }
  tail -1 "$O/prof_backbone.log"
fi
if [ -n "${WITH_EXTRA:-}" ]; then
  timeout -k 10 400 python bench.py --workload scorers > "$O/scorers_bench.json" 2> "$O/scorers_bench.err" || { tail -5 "$O/scorers_bench.err"; exit 1; }
  timeout -k 10 300 python bench.py --workload arxiv --no-cpu-baseline > "$O/arxiv_bench.json" 2> "$O/arxiv_bench.err" || { tail -5 "$O/arxiv_bench.err"; exit 1; }
  timeout -k 10 300 python bench.py --workload rmat --no-cpu-baseline > "$O/rmat_bench.json" 2> "$O/rmat_bench.err" || { tail -5 "$O/rmat_bench.err"; exit 1; }
  echo extra done
fi
