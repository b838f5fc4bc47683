#!/bin/bash
# GPU box: Jaccard parity, then RMAT Jaccard step time per env configuration.
# usage: jac_ab.sh "ENV=V ..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "jaccard or scores_bit_exact or topology or common" > gpurun_out/pytest_jac.log 2>&1 || { tail -30 gpurun_out/pytest_jac.log; exit 1; }
tail -1 gpurun_out/pytest_jac.log
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --workload rmat ${JAC_ARGS:-} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/jac.json 2>gpurun_out/jac.err || { tail -5 gpurun_out/jac.err; exit 1; }
  echo "[$cfg] $(python -c "import json;d=json.load(open('gpurun_out/jac.json'));print(d['ms_per_step'])")"
done
