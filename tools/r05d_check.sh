#!/bin/bash
# Round-5: the fused CG form (compile-time instantiation): ApproxER parity + the T=8
# pins, A/B of the Roman line (GSPARSE_REG_FUSE=0 / 1), then the staged backbone's
# search-geometry variants at N = 4 / 8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05d}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_blas_threads.py \
    -k "approx_er or er_ or cg or roman or blas" -q --maxfail=3 --timeout 600 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
for f in 0 1 0 1; do
  GSPARSE_REG_FUSE=$f timeout -k 10 300 python bench.py --steps 10 --warmup 2 --box-order-steps 0 --no-cpu-baseline \
      > "$OUT/roman_fuse$f.json" 2> "$OUT/roman_fuse$f.err" || { echo "bench rc=$?"; tail -5 "$OUT/roman_fuse$f.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/roman_fuse$f.json'));print('roman fuse=$f ms/step',a['ms_per_step'],a['roofline']['avg_launch_ms'])"
done
timeout -k 10 900 python -u tools/bb_stage_probe.py 18 "0.5,0.8,0.95" "2:512:512;4:512:512;2:1024:256;8:1024:256;2:256:1024" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; tail -5 "$OUT/bb_stage_probe.err"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
