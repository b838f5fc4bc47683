#!/bin/bash
# GPU box: Jaccard parity (R-MAT-22 pin + the Jaccard GPU tests) on the main build, then
# the RMAT bench step of the main build and each variant (libgsparse_V.so), twice each.
# usage: jac_variant_ab.sh TAG V...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
O=gpurun_out/$T
mkdir -p "$O"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmat22.py tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread \
    -k "rmat22 or jaccard or common" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2; do
  for v in main "$@"; do
    if [ "$v" = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
    GSPARSE_LIB=$lib timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err" || { tail -5 "$O/bench_${v}_$rep.err"; exit 1; }
    python3 -c "import json;a=json.load(open('$O/bench_${v}_$rep.json'));print('$v', a['ms_per_step'], a['roofline']['avg_launch_ms'])"
  done
done
echo done
