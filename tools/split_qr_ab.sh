#!/bin/bash
# GPU box: the split form (78 Roman columns in 2 parts) with q in registers (QR=1, the
# default) vs x in registers (GSPARSE_REG_SPLIT_QR=0, needs that build), parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03h_sqr; mkdir -p $O
GSPARSE_REG_SPLIT_QR=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "all_cg_modes or blas_chunks or column_blocks or roman_full or split" > $O/pytest_sqr0.log 2>&1 || { tail -30 $O/pytest_sqr0.log; exit 1; }
tail -1 $O/pytest_sqr0.log
for q in 1 0 1 0; do
  GSPARSE_REG_SPLIT_QR=$q timeout -k 10 200 python tools/cg_probe.py 22662 78 500 8 > $O/p78_q$q.txt 2>&1 || exit 1
  echo "78 cols split QR=$q $(grep solve= $O/p78_q$q.txt)"
done
for q in 1 0; do
  GSPARSE_REG_SPLIT_QR=$q timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_q$q.json 2>$O/bench_q$q.err || exit 1
  python3 -c "import json;a=json.load(open('$O/bench_q$q.json'));print('bench split QR=$q', a['ms_per_step'])"
done
