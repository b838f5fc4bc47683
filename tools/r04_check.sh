#!/bin/bash
# Round-4 check on the GPU box: the pins of what the bench times, the device
# multi-GPU tests, the ApproxER / backbone parity subset, then the default bench line.
# usage: tools/r04_check.sh OUTDIR [extra pytest -k expression]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_distributed.py \
    tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread ${2:+-k "$2"} \
    > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "bench_rc=$?"
