#!/bin/bash
# Round-4 zb: per-thread neighbour-scan cap (64 / 128 / 512) and the deferred-list size
# (256 / 1,024) of the backbone's exact reverse-column certificates; parity of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04zb}
mkdir -p "$OUT"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main c64 c128 b1k c128b1k; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py -x -q \
      --timeout 400 --timeout-method thread -k "reverse_columns or rmat18 or multi_source" > "$OUT/pytest_$v.log" 2>&1 \
      || { echo "pytest $v rc=$?"; tail -20 "$OUT/pytest_$v.log"; exit 1; }
  GSPARSE_LIB=$lib timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_$v.json" 2> "$OUT/bb_$v.err" || exit $?
  echo "$v: $(tail -1 $OUT/pytest_$v.log) $(head -1 $OUT/bb_$v.json)"
done
