#!/bin/bash
# GPU box: backbone parity (goldens, pins, staged parts), the N=1 backbone bench line
# and the staged probe (RMAT-18).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r05o}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "backbone or landmark or staged or geodesic" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python bench.py --workload backbone --steps 3 --warmup 1 --no-cpu-baseline > "$O/bench_backbone.json" 2> "$O/bench_backbone.err" || { tail -20 "$O/bench_backbone.err"; exit 1; }
python3 -c "import json;a=json.load(open('$O/bench_backbone.json'));print('backbone ms/step',a['ms_per_step'])"
timeout -k 10 400 python -u tools/bb_stage_probe.py 18 "0.6,0.9" > "$O/probe.jsonl" 2> "$O/probe.err" || { tail -20 "$O/probe.err"; exit 1; }
python3 - "$O/probe.jsonl" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "summary" in d:
        print(d["summary"])
    else:
        print("N", d["N"], "rank", d["rank_ms"], {k: v for k, v in d["stages_ms"].items()})
PY
echo done
