#!/bin/bash
# GPU box: device normal-stream parity tests, then the RNG kernels' times (bench trace).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-zig}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "device_rng" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench.json" 2> "$O/trace.err" || { tail -5 "$O/trace.err"; exit 1; }
GSPARSE_ZIG_BLOCK=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "device_rng" > "$O/pytest1024.log" 2>&1 || { tail -30 "$O/pytest1024.log"; exit 1; }
tail -1 "$O/pytest1024.log"
grep -E "k_zig|k_project" "$O/trace/run_kernel_stats.csv" | cut -d, -f1,2,4 
