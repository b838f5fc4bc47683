#!/bin/bash
# Round-4 i: 16-lane groups in the 16-source backbone search (parity + A/B vs the
# per-lane form and S = 8), per-part probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04i}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for cfg in "16 1024 1" "16 512 1" "16 1024 0" "8 1024 0"; do
  set -- $cfg
  GSPARSE_BB_MULTI=$1 GSPARSE_BB_THREADS=$2 GSPARSE_BB_GROUPED=$3 GSPARSE_BB_NEARFAR=0 timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_S$1_T$2_g$3.json" 2> "$OUT/bb_S$1_T$2_g$3.err" || exit $?
  echo "S=$1 T=$2 grouped=$3: $(head -1 $OUT/bb_S$1_T$2_g$3.json)"
done
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-1200
