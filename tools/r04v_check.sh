#!/bin/bash
# Round-4 v: margin-stress parity of the backbone's reverse-column decisions, then the
# final rocprofv3 summaries of every bench workload (sources as committed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04v}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    -k "reverse_columns or backbone_rmat12 or multi_source" > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
tools/r04z_profiles.sh "$OUT/prof" roman rmat backbone arxiv || exit $?
