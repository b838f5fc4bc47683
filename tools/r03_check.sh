#!/bin/bash
# GPU box, round 3: the new GPU tests (multi-GPU path, BLAS thread counts, configs[2],
# caller sequences), then the whole suite, the default bench line and a 2-rank
# rehearsal of bench.py --gpus 2 on the one GPU.  usage: r03_check.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r03b}
O=gpurun_out/$T
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_callers.py tests/test_gpu_blas_threads.py tests/test_gpu_arxiv.py -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_new.log" 2>&1 || { tail -60 "$O/pytest_new.log"; exit 1; }
tail -3 "$O/pytest_new.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > "$O/roman_bench.json" 2> "$O/roman_bench.err" || { tail -20 "$O/roman_bench.err"; exit 1; }
cat "$O/roman_bench.json"
GSPARSE_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 1 > "$O/roman_bench_n2_rehearsal.json" 2> "$O/roman_bench_n2_rehearsal.err" || { tail -20 "$O/roman_bench_n2_rehearsal.err"; exit 1; }
cat "$O/roman_bench_n2_rehearsal.json"
