#!/bin/bash
# Round-5: the CG back to the unfused form (Roman line), the staged backbone with the
# N >= 4 search geometry under several phase schedules, its GPU tests, and the drop-in
# API timers (Roman Jaccard+ApproxER, R-MAT-22 Jaccard-T).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05e}
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --box-order-steps 0 --no-cpu-baseline \
    > "$OUT/roman.json" 2> "$OUT/roman.err" || { echo "bench rc=$?"; tail -5 "$OUT/roman.err"; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/roman.json'));print('roman ms/step',a['ms_per_step'],a['roofline']['avg_launch_ms'])"
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py -k "staged or gloo" -q --maxfail=3 --timeout 600 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 900 python -u tools/bb_stage_probe.py 18 "0.5,0.8,0.95;0.3,0.6,0.85,0.95;0.6,0.9;0.7,0.9,0.97;0.4,0.7,0.9,0.97,0.99" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; tail -5 "$OUT/bb_stage_probe.err"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
timeout -k 10 300 python tools/api_timer.py > "$OUT/api_roman.json" 2> "$OUT/api_roman.err" || { echo "api rc=$?"; tail -5 "$OUT/api_roman.err"; exit 1; }
cat "$OUT/api_roman.json"
timeout -k 10 300 python tools/api_timer.py rmat > "$OUT/api_rmat.json" 2> "$OUT/api_rmat.err" || { echo "api rmat rc=$?"; tail -5 "$OUT/api_rmat.err"; exit 1; }
cat "$OUT/api_rmat.json"
