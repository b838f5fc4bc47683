#!/bin/bash
# Round-5: the CG's bank-aligned diagonal slots -- the ApproxER parity subset, the T=8
# pins, the Roman line (against 207.5 ms per solve unaligned, r05e).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05f}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_blas_threads.py \
    -k "approx_er or er_ or cg or roman or blas" -q --maxfail=3 --timeout 600 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -2 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --box-order-steps 0 --no-cpu-baseline \
    > "$OUT/roman$i.json" 2> "$OUT/roman$i.err" || { echo "bench rc=$?"; tail -5 "$OUT/roman$i.err"; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/roman$i.json'));print('roman ms/step',a['ms_per_step'],a['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d "$OUT/sq" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline > "$OUT/bench_sq.json" 2> "$OUT/sq.err" || { echo "pmc rc=$?"; exit 1; }
python3 tools/pmc_summary.py --calls=1 "$OUT/sq_summary.json" "$OUT/sq" | grep regwide
