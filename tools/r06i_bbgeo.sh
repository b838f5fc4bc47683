#!/bin/bash
# Per-rank search geometry at N = 4 / 8 under the current phases: S sources per
# workgroup : threads : slabs (bb_stage_probe.py variants)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06i
mkdir -p "$OUT"
timeout -k 10 900 python -u tools/bb_stage_probe.py 18 "0.6,0.85" "2:1024:256;4:1024:256;4:512:512;8:512:512;2:512:512" \
    > "$OUT/geo.jsonl" 2> "$OUT/geo.err" || exit $?
tail -1 "$OUT/geo.jsonl"
