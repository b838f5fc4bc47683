#!/bin/bash
# Round-5: the candidate top-k -- its GPU tests (goldens, specials, the R-MAT-22 pin),
# the R-MAT-22 Jaccard-T line, one rank's share probe of the current Jaccard.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05i}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rmat22.py tests/test_gpu_distributed.py \
    tests/test_gpu_callers.py -k "topk or rmat22 or sparsify or gloo or nccl or mask or caller" -q --maxfail=3 --timeout 800 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|assert" "$OUT/pytest.log" | head -20; exit 1; }
for m in 12 8; do
  if [ $m = 8 ]; then export GSPARSE_TOPK=8; else unset GSPARSE_TOPK; fi
  timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/rmat_topk$m.json" 2> "$OUT/rmat_topk$m.err" || { echo "rmat rc=$?"; tail -5 "$OUT/rmat_topk$m.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/rmat_topk$m.json'));print('rmat topk$m ms/step',a['ms_per_step'],a['kernels'].get('jaccard'),a['kernels'].get('topk'))"
done
unset GSPARSE_TOPK
timeout -k 10 600 python tools/shares_probe.py 22 3 > "$OUT/shares_probe.json" 2> "$OUT/shares_probe.err" || { echo "probe rc=$?"; tail -5 "$OUT/shares_probe.err"; exit 1; }
tail -1 "$OUT/shares_probe.json" | cut -c1-1500
