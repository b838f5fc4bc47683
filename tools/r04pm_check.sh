#!/bin/bash
# Round-4 pm: backbone part of a pair by its higher-degree endpoint (min id) vs the
# lower-degree one (max id, default): per-part probe of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04pm}
mkdir -p "$OUT"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
GSPARSE_LIB=$PKG/libgsparse_pmin.so timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe_pmin.json" 2> "$OUT/bb_probe_pmin.err" || exit $?
tail -1 "$OUT/bb_probe_pmin.json" | cut -c1-1500
