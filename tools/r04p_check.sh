#!/bin/bash
# Round-4 p: backbone with ascending-degree batch order as the default: parity, the
# bench line, per-part probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04p}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_boundary.py tests/test_gpu_distributed.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 400 python bench.py --workload backbone --steps 3 --warmup 1 > "$OUT/bench_backbone.json" 2> "$OUT/bench_backbone.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_backbone.json'));print('backbone ms/step',a['ms_per_step'],a.get('cpu_baseline'))"
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-1500
