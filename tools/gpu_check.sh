#!/bin/bash
# GPU box: parity tests (optionally filtered) then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K=${1:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.log
exit $rc
