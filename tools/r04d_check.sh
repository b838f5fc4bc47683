#!/bin/bash
# Round-4 d: parity (pins, mode 5, exact-ER kept sets, multi-GPU top-k), p-update group
# A/B (GS_PGRP variants), R-MAT-22 Jaccard-T, backbone parts with phases, N=2 rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04c}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py tests/test_gpu_distributed.py \
    -x -q --timeout 300 --timeout-method thread \
    -k "pins or all_cg_modes or blas_chunks or column_blocks or roman_full or split_tail or jaccard or rmat14 or nccl or gloo or exact_er or backbone" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main kp2 pg8; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  [ -f "$lib" ] || continue
  GSPARSE_LIB=$lib GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$OUT/probe_$v.txt" 2>&1 || exit $?
  echo "$v: $(tail -1 $OUT/probe_$v.txt)"
  GSPARSE_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --box-order-steps 0 > "$OUT/bench_$v.json" 2> "$OUT/bench_$v.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/bench_$v.json'));print('$v roman ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
done
timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat.json" 2> "$OUT/rmat.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/rmat.json'));print('rmat ms/step',a['ms_per_step'],a['kernels'])"
timeout -k 10 400 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-900
tools/rehearse_ranks.sh r04c_ranks 2
