#!/bin/bash
# GPU box: landmark searches spread over the GPU (k_lm_round) vs one workgroup per
# landmark: parity tests, then the staged backbone probe under both (RMAT-18).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05m
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_pins.py -m gpu -x -v --timeout 300 --timeout-method thread \
    -k "landmark or staged or backbone" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for coop in 1 0; do
  GSPARSE_BB_LMCOOP=$coop timeout -k 10 400 python -u tools/bb_stage_probe.py 18 "0.6,0.9" > "$O/probe_coop$coop.jsonl" 2> "$O/probe_coop$coop.err" || { tail -20 "$O/probe_coop$coop.err"; exit 1; }
  python3 - "$O/probe_coop$coop.jsonl" "$coop" <<'EOF'
import json, sys
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "summary" in d:
        print("coop", sys.argv[2], d["summary"])
    else:
        print("coop", sys.argv[2], "N", d["N"], "begin", d["stages_ms"]["begin"], "rank", d["rank_ms"])
EOF
done
echo done
