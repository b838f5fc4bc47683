#!/bin/bash
# Round-4 r: software-pipelined Jaccard probe loop (list loads of the next step in
# flight during this step's probes): parity, RMAT-22 A/B, shares probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04r}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py tests/test_gpu_arxiv.py \
    -x -q --timeout 300 --timeout-method thread -k "jaccard or scores_bit_exact or rmat14" \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main p0 p8 p11 main p0; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat_$v.json" 2> "$OUT/rmat_$v.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/rmat_$v.json'));print('$v rmat ms/step',a['ms_per_step'],a['kernels'])"
done
GSPARSE_JAC_CONCURRENT=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_serial" -o rmat -- python3 bench.py --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/rmat_serial.json" 2> "$OUT/rmat_serial.err" || exit $?
timeout -k 10 500 python tools/shares_probe.py 22 2 > "$OUT/shares.json" 2> "$OUT/shares.err" || exit $?
tail -1 "$OUT/shares.json" | cut -c1-300
