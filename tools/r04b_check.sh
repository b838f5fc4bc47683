#!/bin/bash
# Round-4 b: mode-5 parity subset + pins on the current build, the default bench line,
# the R-MAT-22 Jaccard-T line (top-k in the step) and the backbone per-rank probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04b}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py tests/test_gpu_distributed.py \
    -x -q --timeout 300 --timeout-method thread \
    -k "pins or all_cg_modes or blas_chunks or column_blocks or roman_full or split_tail or jaccard or rmat14 or nccl or gloo" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$OUT/probe.txt" 2>&1 || exit $?
tail -2 "$OUT/probe.txt"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench.json'));print('roman ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat.json" 2> "$OUT/rmat.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/rmat.json'));print('rmat ms/step',a['ms_per_step'],a['kernels'])"
timeout -k 10 400 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-600
# A/B: the round-3 slot code (libgsparse_v1.so: -DGS_CG_V2=0 in the whole-column kernels)
V1=$PWD/gnn-sparsification-research_amd/gsparse/libgsparse_v1.so
if [ -f "$V1" ]; then
  GSPARSE_LIB=$V1 GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$OUT/probe_v1.txt" 2>&1 || exit $?
  tail -2 "$OUT/probe_v1.txt"
  GSPARSE_LIB=$V1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --box-order-steps 0 > "$OUT/bench_v1.json" 2> "$OUT/bench_v1.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/bench_v1.json'));print('v1 roman ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
fi
