#!/bin/bash
# A/B: Jaccard probe lists from a 3-byte packed copy of the indices (GS_JAC_IX3=1
# variant library) vs the default 4-byte lists; parity of the variant first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04ix3}
mkdir -p "$OUT"
V=$PWD/gnn-sparsification-research_amd/gsparse/libgsparse_ix3.so
GSPARSE_LIB=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_arxiv.py tests/test_gpu_distributed.py -k "jaccard or Jaccard or common" > "$OUT/parity.log" 2>&1 || { echo "parity rc=$?"; tail -20 "$OUT/parity.log"; exit 1; }
tail -1 "$OUT/parity.log"
for v in base ix3 base ix3; do
  if [ $v = ix3 ]; then export GSPARSE_LIB=$V; else unset GSPARSE_LIB; fi
  timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/$v.json" 2> "$OUT/$v.err" || { echo "$v rc=$?"; tail -5 "$OUT/$v.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/$v.json').read().strip().splitlines()[-1]);print('$v',a['ms_per_step'],'ms/step',a.get('jaccard_ms') or '')"
done
