#!/bin/bash
# Round-4 j: backbone search workgroup shape A/B at 16 sources (1 x 1024, 2 x 512,
# 4 x 256 threads per CU), and the Jaccard per-rank probe with warmed plans.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04j}
mkdir -p "$OUT"
for cfg in "16 1024 256" "16 512 512" "16 256 1024" "8 512 512"; do
  set -- $cfg
  GSPARSE_BB_MULTI=$1 GSPARSE_BB_THREADS=$2 GSPARSE_BB_SLABS=$3 GSPARSE_BB_NEARFAR=0 timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_S$1_T$2_W$3.json" 2> "$OUT/bb_S$1_T$2_W$3.err" || exit $?
  echo "S=$1 T=$2 slabs=$3: $(head -1 $OUT/bb_S$1_T$2_W$3.json)"
done
timeout -k 10 500 python tools/shares_probe.py 22 2 > "$OUT/shares.json" 2> "$OUT/shares.err" || exit $?
tail -1 "$OUT/shares.json" | cut -c1-1500
