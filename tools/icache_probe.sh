#!/bin/bash
# GPU box: instruction-cache behaviour of the register-resident CG (Roman size, 256
# columns x 100 iterations): lists the SQC counters, then one --pmc pass per pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-icache}
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
grep -io "SQC_[A-Z0-9_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT_INST[A-Z_]*\|SQ_INST_[A-Z_]*" $O/avail.txt | sort -u > $O/sqc_names.txt || true
cat $O/sqc_names.txt | tr '\n' ' '; echo
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  GSPARSE_CG_MODE=5 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/cg_probe.py 22662 256 100 8 > $O/p$i.log 2>&1 || { echo "pass failed: $set"; tail -5 $O/p$i.log; continue; }
  tail -1 $O/p$i.log
done
python3 tools/pmc_summary.py $O/summary.json $O/p1 $O/p2 $O/p3 > /dev/null 2>&1
python3 - $O/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    if "regwide" in k:
        print(k, json.dumps(v))
PY
