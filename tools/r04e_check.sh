#!/bin/bash
# Round-4 e: 16-bit quotient Jaccard tables -- parity (every row class, 16- and 22-bit
# ids, forced overflow), R-MAT-22 Jaccard-T A/B (main = classes 1-3, q16c3 = class 3
# only, q16off = int32 tables), per-kernel trace, per-rank shares probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04e}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_arxiv.py \
    -x -q --timeout 300 --timeout-method thread -k "jaccard or scores_bit_exact or rmat14" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main q16c3 q16off; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  [ -f "$lib" ] || continue
  GSPARSE_LIB=$lib timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat_$v.json" 2> "$OUT/rmat_$v.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/rmat_$v.json'));print('$v rmat ms/step',a['ms_per_step'],a['kernels'])"
done
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o rmat -- python3 bench.py --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/rmat_prof.json" 2> "$OUT/rmat_prof.err" || exit $?
timeout -k 10 500 python tools/shares_probe.py 22 2 > "$OUT/shares.json" 2> "$OUT/shares.err" || exit $?
tail -1 "$OUT/shares.json" | cut -c1-1200
