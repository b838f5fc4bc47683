#!/bin/bash
# GPU box: multi-source backbone parity, then RMAT-18 / Roman backbone timings per S.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "backbone" > gpurun_out/pytest_bb.log 2>&1 || { tail -30 gpurun_out/pytest_bb.log; exit 1; }
tail -1 gpurun_out/pytest_bb.log
for S in ${BB_S:-1 2 4 8}; do
  GSPARSE_BB_MULTI=$S timeout -k 10 300 python bench.py --workload backbone --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bbm.json 2>gpurun_out/bbm.err || { tail -5 gpurun_out/bbm.err; exit 1; }
  echo "S=$S rmat18 $(python -c "import json;d=json.load(open('gpurun_out/bbm.json'));print(d['ms_per_step'], d['config']['kept'], d['roofline']['relaxations_per_launch_rank0'])")"
done
