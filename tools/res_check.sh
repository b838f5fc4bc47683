#!/bin/bash
# GPU box: the ApproxER parity cases of every CG mode, then the default line's
# resident-solver phase clock and step time (twice).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "blas_chunks or column_blocks or all_cg_modes or approx_er" > gpurun_out/pytest_res.log 2>&1 || { tail -30 gpurun_out/pytest_res.log; exit 1; }
tail -1 gpurun_out/pytest_res.log
for r in 1 2; do
  GSPARSE_RES_PROF=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/b3.json 2>gpurun_out/b3.err || exit 1
  echo "$(grep -i resident gpurun_out/b3.err | tail -1 | cut -c40-) $(python -c "import json;d=json.load(open('gpurun_out/b3.json'));print(d['ms_per_step'])")"
done
