#!/bin/bash
# Round-5 first GPU pass: the new full-size pins (configs[3] R-MAT-22, configs[2]
# arxiv geometry), the whole GPU suite, smoke, the default bench line, the Roman
# profile (counters of the timed T=8 call only), the arxiv line with its CPU baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05a}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 900 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_roman.json'));print('roman ms/step',a['ms_per_step'])"
tools/profile_bench.sh "$OUT/prof_roman" --workload roman || { echo "profile rc=$?"; exit 1; }
timeout -k 10 600 python bench.py --workload arxiv > "$OUT/bench_arxiv.json" 2> "$OUT/bench_arxiv.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_arxiv.json'));print('arxiv ms/step',a['ms_per_step'], a['cpu_baseline']['value'])"
