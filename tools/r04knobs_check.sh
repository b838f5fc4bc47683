#!/bin/bash
# Round-4 knobs: the backbone's landmark count and sources per workgroup (with the
# near-far order at 8) on the final code, RMAT-18 whole prune.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04knobs}
mkdir -p "$OUT"
run() {
  env "$@" timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb.json" 2> "$OUT/bb.err" || exit $?
  echo "$*: $(head -1 $OUT/bb.json)"
}
run GSPARSE_BB_LANDMARKS=48
run GSPARSE_BB_NEARFAR=1
run GSPARSE_BB_NEARFAR=3
run GSPARSE_BB_LANDMARKS=96
run GSPARSE_BB_LANDMARKS=32
run GSPARSE_BB_SLABS=768
run GSPARSE_BB_THREADS=256 GSPARSE_BB_SLABS=1024
run GSPARSE_BB_MULTI=4
