#!/bin/bash
# Round-5: the fused CG p update, the remainder-sized Jaccard list steps and the staged
# backbone.  GPU tests first (the whole suite), then A/B bench lines (fused p update
# off / on; Jaccard-T), the staged backbone line and its per-rank probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05c}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 900 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
for f in 0 1; do
  GSPARSE_REG_FUSE=$f timeout -k 10 300 python bench.py --steps 10 --warmup 2 --box-order-steps 0 --no-cpu-baseline \
      > "$OUT/roman_fuse$f.json" 2> "$OUT/roman_fuse$f.err" || { echo "bench rc=$?"; tail -5 "$OUT/roman_fuse$f.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$OUT/roman_fuse$f.json'));print('roman fuse=$f ms/step',a['ms_per_step'],a['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/rmat.json" 2> "$OUT/rmat.err" || { echo "rmat rc=$?"; tail -5 "$OUT/rmat.err"; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/rmat.json'));print('rmat ms/step',a['ms_per_step'],a['kernels'].get('jaccard'), a.get('dropin_numpy_tie_break'))"
timeout -k 10 300 python bench.py --workload backbone --no-cpu-baseline > "$OUT/backbone.json" 2> "$OUT/backbone.err" || { echo "bb rc=$?"; tail -5 "$OUT/backbone.err"; exit 1; }
python3 -c "import json;a=json.load(open('$OUT/backbone.json'));print('backbone ms/step',a['ms_per_step'])"
timeout -k 10 600 python -u tools/bb_stage_probe.py 18 "0.5,0.8,0.95;0.25,0.5,0.75,0.9,0.97;0.9;;0.6,0.85,0.95,0.99" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; tail -5 "$OUT/bb_stage_probe.err"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
