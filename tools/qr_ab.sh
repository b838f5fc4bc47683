#!/bin/bash
# GPU box: mode-5 parity subset, then q-in-registers (GSPARSE_REG_QR=1) vs
# q-recomputed (0): CG probe per column-iteration and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-qr}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "all_cg_modes or blas_chunks or column_blocks or roman_full" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for q in 1 0; do
  GSPARSE_REG_QR=$q GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$O/probe_q$q.txt" 2>&1 || { tail -20 "$O/probe_q$q.txt"; exit 1; }
  echo "QR=$q"; grep -v "^\s*$" "$O/probe_q$q.txt" | tail -3
done
for q in 1 0; do
  GSPARSE_REG_QR=$q timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_q$q.json" 2> "$O/bench_q$q.err" || { tail -20 "$O/bench_q$q.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$O/bench_q$q.json'));print('QR=$q ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
done
