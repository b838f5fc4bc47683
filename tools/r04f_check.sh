#!/bin/bash
# Round-4 f: near-far backbone searches (parity + step sweep on RMAT-18 + per-part probe),
# Jaccard probe loop without masked-off steps (parity, R-MAT-22 bench, per-class trace,
# per-rank shares).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04f}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pins.py tests/test_gpu_boundary.py \
    -x -q --timeout 400 --timeout-method thread -k "backbone or jaccard or scores_bit_exact" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for f in 0 0.25 0.5 1 2; do
  GSPARSE_BB_NEARFAR=$f timeout -k 10 200 python tools/bb_probe.py 18 1 whole > "$OUT/bb_nf_$f.json" 2> "$OUT/bb_nf_$f.err" || exit $?
  echo "nearfar $f: $(head -1 $OUT/bb_nf_$f.json)"
done
timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat.json" 2> "$OUT/rmat.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/rmat.json'));print('rmat ms/step',a['ms_per_step'],a['kernels'])"
GSPARSE_JAC_CONCURRENT=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_serial" -o rmat -- python3 bench.py --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/rmat_serial.json" 2> "$OUT/rmat_serial.err" || exit $?
timeout -k 10 500 python tools/shares_probe.py 22 2 > "$OUT/shares.json" 2> "$OUT/shares.err" || exit $?
tail -1 "$OUT/shares.json" | cut -c1-1200
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-900
