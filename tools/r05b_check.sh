#!/bin/bash
# Round-5 staged metric backbone: the backbone GPU tests (single call, parts on
# separate contexts, gloo ranks sharing the GPU), the bench line, and the per-rank
# probe of the staged multi-rank form on R-MAT-18.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_pins.py tests/test_gpu_boundary.py \
    tests/test_gpu_parity.py -k "backbone or gloo or staged or nccl or boundary" -q --maxfail=3 --timeout 600 \
    --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python bench.py --workload backbone --no-cpu-baseline > "$OUT/bench_backbone.json" 2> "$OUT/bench_backbone.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench_backbone.err"; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/bench_backbone.json'));print('backbone ms/step',a['ms_per_step'])"
timeout -k 10 600 python -u tools/bb_stage_probe.py 18 "0.5,0.8,0.95;0.25,0.5,0.75,0.9,0.97;0.9;;0.6,0.85,0.95,0.99" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; tail -5 "$OUT/bb_stage_probe.err"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
