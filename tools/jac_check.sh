#!/bin/bash
# GPU box: Jaccard parity tests, RMAT-22 bench line, per-kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "jaccard or rmat14 or scores_bit_exact or roman_full_structural or edge_cases" > gpurun_out/pj.log 2>&1 || { tail -30 gpurun_out/pj.log; exit 1; }
tail -1 gpurun_out/pj.log
timeout -k 10 400 python bench.py --workload rmat --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/brmat.log 2> gpurun_out/brmat.err || exit 1
cut -c1-200 gpurun_out/brmat.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_jac -o run -- python3 bench.py --workload rmat --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_jac.log 2>&1 || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open('gpurun_out/prof_jac/run_kernel_stats.csv')):
    if 'jac' in r['Name']:
        print(r['Name'].split('(')[0][:40], r['Calls'], round(float(r['AverageNs'])/1e6, 3))
PY
