#!/bin/bash
# Round-4 w: 6-entry SpMV for slots of short rows in the register-resident CG (V2):
# mode-5 parity incl. the full-Roman pins, CG probe and bench A/B against the 8-entry form.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04w}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py tests/test_gpu_blas_threads.py \
    -x -q --timeout 400 --timeout-method thread -k "pins or all_cg_modes or blas_chunks or column_blocks or roman_full or split_tail or approx_er" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main w8 main w8; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$OUT/probe_$v.txt" 2>&1 || exit $?
  echo "$v: $(tail -1 $OUT/probe_$v.txt)"
  GSPARSE_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --box-order-steps 0 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/bench_$v.json'));print('$v roman ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
done
