#!/bin/bash
# Round-5: top-k with wave-aggregated compaction -- tests and the R-MAT-22 line (A/B vs 8-bit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05j}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rmat22.py -k "topk or rmat22" -q --maxfail=3 \
    --timeout 800 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|assert" "$OUT/pytest.log" | head -20; exit 1; }
for m in 12 8; do
  if [ $m = 8 ]; then export GSPARSE_TOPK=8; else unset GSPARSE_TOPK; fi
  GSPARSE_TOPK_DEBUG=1 timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/rmat_topk$m.json" 2> "$OUT/rmat_topk$m.err" || { echo "rmat rc=$?"; tail -5 "$OUT/rmat_topk$m.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/rmat_topk$m.json'));print('rmat topk$m ms/step',a['ms_per_step'],a['kernels'].get('jaccard'),a['kernels'].get('topk'))"
done
grep -m2 "\[topk\]" "$OUT/rmat_topk12.err"
