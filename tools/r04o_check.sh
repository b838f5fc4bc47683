#!/bin/bash
# Round-4 o: backbone batch order (descending / ascending column count) and the
# neighbour-scan cap of the exact reverse-column certificate; parity of the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04o}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main xdeg4k xdeginf; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  for o in desc asc; do
    GSPARSE_LIB=$lib GSPARSE_BB_ORDER=$o timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_${v}_$o.json" 2> "$OUT/bb_${v}_$o.err" || exit $?
    echo "$v order=$o: $(head -1 $OUT/bb_${v}_$o.json)"
  done
done
GSPARSE_BB_ORDER=asc timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" > "$OUT/pytest_asc.log" 2>&1 || { echo "pytest asc rc=$?"; tail -30 "$OUT/pytest_asc.log"; exit 1; }
tail -1 "$OUT/pytest_asc.log"
