#!/bin/bash
# Round-5 final: the whole GPU suite, smoke(), the default bench line (with its CPU
# baseline), then the rocprofv3 summaries of the four workloads on these sources, the
# secondary bench lines with their CPU baselines, and the staged backbone probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${1:-gpurun_out/r05final}
mkdir -p "$OUT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 900 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -1 "$OUT/pytest.log"
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)" "$OUT/pytest.log" | head -20; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { echo "smoke rc=$?"; tail -20 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_roman.json" 2> "$OUT/bench_roman.err" || exit $?
python3 -c "import json;a=json.load(open('$OUT/bench_roman.json'));print('roman ms/step',a['ms_per_step'],a['cpu_baseline']['value'])"
for wl in roman rmat backbone arxiv; do
  tools/profile_bench.sh "$OUT/prof_$wl" --workload $wl || { echo "profile $wl rc=$?"; exit 1; }
  echo "$wl profiled"
done
for wl in rmat backbone arxiv scorers; do
  timeout -k 10 600 python bench.py --workload $wl > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { echo "$wl rc=$?"; tail -5 "$OUT/bench_$wl.err"; exit 1; }
  python3 -c "import json;a=json.loads(open('$OUT/bench_$wl.json').read().strip().splitlines()[-1]);print('$wl',a['ms_per_step'],'ms/step', (a.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 300 python tools/api_timer.py > "$OUT/api_roman.json" 2> "$OUT/api_roman.err" || exit $?
timeout -k 10 300 python tools/api_timer.py rmat > "$OUT/api_rmat.json" 2> "$OUT/api_rmat.err" || exit $?
timeout -k 10 900 python -u tools/bb_stage_probe.py 18 "0.6,0.9;0.5,0.8,0.95;" > "$OUT/bb_stage_probe.jsonl" 2> "$OUT/bb_stage_probe.err" || { echo "probe rc=$?"; exit 1; }
tail -1 "$OUT/bb_stage_probe.jsonl"
