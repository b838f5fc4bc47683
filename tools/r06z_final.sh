#!/bin/bash
# Round-6 final: the whole GPU suite, smoke(), the default bench line (CPU baseline
# included), the rocprofv3 summaries of the four workloads on these sources, and the
# secondary bench lines.  usage: r06z_final.sh [OUT]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r06z}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 900 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -1 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_roman.json'));print('roman ms/step',a['ms_per_step'],'box order',a.get('box_blas_order',{}).get('ms_per_step'),'cpu',a['cpu_baseline']['value'])"
