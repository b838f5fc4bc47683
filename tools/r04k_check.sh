#!/bin/bash
# Round-4 k: fire-and-forget label atomics in the multi-source backbone search
# (parity + A/B against the returning form), per-part probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04k}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main noret0; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  for S in 16 8; do
    GSPARSE_LIB=$lib GSPARSE_BB_MULTI=$S timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_${v}_S$S.json" 2> "$OUT/bb_${v}_S$S.err" || exit $?
    echo "$v S=$S: $(head -1 $OUT/bb_${v}_S$S.json)"
  done
done
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-1200
