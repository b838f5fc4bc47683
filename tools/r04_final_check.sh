#!/bin/bash
# Round-4 final: the whole GPU suite, smoke(), the default bench line, then the
# rocprofv3 summaries of every bench workload on these sources.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r04final}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_roman.json'));print('roman ms/step',a['ms_per_step'])"
tools/r04z_profiles.sh "$OUT/prof" roman rmat backbone arxiv || exit $?
timeout -k 10 600 python tools/bb_probe.py 18 1 > "$OUT/bb_probe.json" 2> "$OUT/bb_probe.err" || exit $?
tail -1 "$OUT/bb_probe.json" | cut -c1-1500
