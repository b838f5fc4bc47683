#!/bin/bash
# GPU box: mode-5 parity subset, then the CG probe for each GSPARSE_* setting given
# ("-" = defaults).  usage: m5_ab.sh TAG CFG...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1
O=gpurun_out/$T
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "all_cg_modes or blas_chunks or column_blocks or roman_full" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
shift
bash tools/probe_ab.sh "$T" "$@"
