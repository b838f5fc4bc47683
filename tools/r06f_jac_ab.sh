#!/bin/bash
# round 6: Jaccard tables with the 24-bit multiplicative hash and the packed-minimum
# bucket test (main) against the round-5 form (libgsparse_jold.so): Jaccard parity and
# the full-size R-MAT-22 pins on main, then the R-MAT-22 Jaccard-T step for both,
# interleaved twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06f
mkdir -p "$O"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "jaccard or scores_bit_exact or topology or common" > "$O/pytest_jac.log" 2>&1 || { tail -30 "$O/pytest_jac.log"; exit 1; }
tail -1 "$O/pytest_jac.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmat22.py -m gpu -x -q --timeout 500 --timeout-method thread > "$O/pytest_rmat22.log" 2>&1 || { tail -30 "$O/pytest_rmat22.log"; exit 1; }
tail -1 "$O/pytest_rmat22.log"
for rep in 1 2; do
  for v in main jold; do
    lib=$PKG/libgsparse.so; [ $v = main ] || lib=$PKG/libgsparse_$v.so
    GSPARSE_LIB=$lib timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$O/rmat_${v}_$rep.json" 2> "$O/rmat_${v}_$rep.err" || { tail -5 "$O/rmat_${v}_$rep.err"; exit 1; }
    python3 -c "import json;d=json.load(open('$O/rmat_${v}_$rep.json'));print('$v rep $rep ms/step',d['ms_per_step'],'jaccard ms',round(d['kernels']['jaccard']['ms']/d['kernels']['jaccard']['launches'],3))"
  done
done
