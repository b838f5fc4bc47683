#!/bin/bash
# round 6: the backbone full-mask pins with decision classes, the distributed Jaccard-T
# select, and the existing backbone / distributed tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R06A_TAG:-r06a}
mkdir -p "$O"
T="timeout -k 10"
PT="python -u -m pytest -x -v -s --timeout 300 --timeout-method thread"
$T 600 $PT tests/test_gpu_backbone_pins.py > "$O/pins.log" 2>&1 || { tail -40 "$O/pins.log"; exit 1; }
grep -E "decision classes|R-MAT-18:|passed|failed|skipped" "$O/pins.log"
$T 600 $PT tests/test_gpu_distributed.py > "$O/dist.log" 2>&1 || { tail -40 "$O/dist.log"; exit 1; }
tail -2 "$O/dist.log"
$T 600 python -u -m pytest tests -m gpu -k "backbone or Backbone or boundary" -x -q --timeout 300 --timeout-method thread > "$O/bb_tests.log" 2>&1 || { tail -40 "$O/bb_tests.log"; exit 1; }
tail -2 "$O/bb_tests.log"
