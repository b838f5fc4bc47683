#!/bin/bash
# Round-4 x: backbone batches from a global counter (dynamic) vs static striding:
# parity, RMAT-18 timing both ways, per-part probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04x}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for x in 1 0 1 0; do
  GSPARSE_BB_DYNAMIC=$x timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_dyn$x.json" 2> "$OUT/bb_dyn$x.err" || exit $?
  echo "dynamic=$x: $(head -1 $OUT/bb_dyn$x.json)"
done
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-1500
