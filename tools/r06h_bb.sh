#!/bin/bash
# Backbone begin without atomics / host partial sort: the full-mask pins, the backbone
# parity tests, the bench line and the N-rank stage probe (one schedule)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06h
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_backbone_pins.py tests/test_gpu_parity.py tests/test_gpu_pins.py \
    tests/test_gpu_distributed.py -m gpu -q -k "backbone or bb" -s --timeout 500 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -1 "$OUT/pytest.log"
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head; exit 1; }
timeout -k 10 300 python bench.py --workload backbone --steps 5 --warmup 2 > "$OUT/bench_backbone.json" 2> "$OUT/bench_backbone.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_backbone.json'));print('backbone ms/step',a['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload backbone --steps 3 --warmup 1 > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u tools/bb_stage_probe.py 18 "0.6,0.85" > "$OUT/stage_probe.jsonl" 2> "$OUT/stage_probe.err" || exit $?
tail -1 "$OUT/stage_probe.jsonl"
