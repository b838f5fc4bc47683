#!/bin/bash
# A/B: Jaccard probe lists read by unconditional 64-lane steps from a scalar base
# (the committed sources under test) vs the previous masked per-element loads
# (libgsparse_base.so, the last validated build); parity of the new build first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04ul}
mkdir -p "$OUT"
B=$PWD/gnn-sparsification-research_amd/gsparse/libgsparse_base.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_arxiv.py tests/test_gpu_distributed.py tests/test_gpu_boundary.py -k "jaccard or Jaccard or common" > "$OUT/parity.log" 2>&1 || { echo "parity rc=$?"; tail -20 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
for v in base new base new; do
  if [ $v = base ]; then export GSPARSE_LIB=$B; else unset GSPARSE_LIB; fi
  timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v rc=$?"; tail -5 "$OUT/$v.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]);print('$v',a['ms_per_step'],'ms/step')"
done
