#!/bin/bash
# round 6: A/B of the stored-q register CG (GS_CG_QS) against the main build, plus the
# T = 8 full-size pins on the variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06b
mkdir -p "$O"
PKG=gnn-sparsification-research_amd/gsparse
bash tools/variant_ab.sh r06b qs main || exit 1
GSPARSE_LIB=$PWD/$PKG/libgsparse_qs.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pins.py -x -q --timeout 300 --timeout-method thread -k roman > "$O/pins_qs.log" 2>&1 || { tail -30 "$O/pins_qs.log"; exit 1; }
tail -1 "$O/pins_qs.log"
