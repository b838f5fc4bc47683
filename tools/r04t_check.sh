#!/bin/bash
# Round-4 t: the whole GPU suite on the current sources, the default bench line,
# and the Jaccard pipelining A/B (GS_JAC_PIPE masks 0x9 default, 0, 0x8, 0xB).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04t}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python bench.py > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_roman.json'));print('roman ms/step',a['ms_per_step'],a['roofline']['on_chip'] if 'on_chip' in a['roofline'] else '')"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
for v in main p0 p8 p11 main p0; do
  if [ $v = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib timeout -k 10 400 python bench.py --workload rmat --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/rmat_$v.json" 2> "$OUT/rmat_$v.err" || exit $?
  python3 -c "import json;a=json.load(open('$OUT/rmat_$v.json'));print('$v rmat ms/step',a['ms_per_step'],a['kernels'])"
done
