#!/bin/bash
# GPU box: mode-5 parity subset (split variants included), then the default bench
# line with the split tail and without it (GSPARSE_REG_SPLIT=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-split}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "all_cg_modes or blas_chunks or column_blocks or roman_full" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for sp in auto 0; do
  if [ $sp = auto ]; then unset GSPARSE_REG_SPLIT; else export GSPARSE_REG_SPLIT=$sp; fi
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_$sp.json" 2> "$O/bench_$sp.err" || { tail -20 "$O/bench_$sp.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$O/bench_$sp.json'));print('split=$sp ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
done
