#!/bin/bash
# Round-4 u: chunked probing in the 16K / 32K quotient classes (parity, RMAT-22 A/B
# against per-entry probing, per-class serial trace, shares probe).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04u}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_arxiv.py \
    -x -q --timeout 300 --timeout-method thread -k "jaccard or scores_bit_exact or rmat14" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for x in 1 0 1 0; do
  GSPARSE_JAC_CHUNKED=$x timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat_c$x.json" 2> "$OUT/rmat_c$x.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/rmat_c$x.json'));print('chunked=$x rmat ms/step',a['ms_per_step'],a['kernels'])"
done
GSPARSE_JAC_CONCURRENT=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_serial" -o rmat -- python3 bench.py --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/rmat_serial.json" 2> "$OUT/rmat_serial.err" || exit $?
timeout -k 10 500 python tools/shares_probe.py 22 2 > "$OUT/shares.json" 2> "$OUT/shares.err" || exit $?
tail -1 "$OUT/shares.json" | cut -c1-300
