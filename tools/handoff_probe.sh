#!/bin/bash
# GPU box: cost of the split CG's hand-offs.  78 Roman columns (the N = 8 rank's tail)
# in 2 parts, kernel trace of the split launch with the hand-offs (spin budget as
# shipped) and without them (GSPARSE_REG_SPLIT_SPIN=0: every part gives up at once and
# its hand-offs become plain barriers -- results discarded, the host re-solves whole).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-handoff}
mkdir -p "$O"
for spin in ship 0; do
  env=""; [ $spin = 0 ] && env="GSPARSE_REG_SPLIT_SPIN=0"
  env GSPARSE_REG_SPLIT=2 $env timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/t_$spin" -o run -- \
      python3 tools/cg_probe.py 22662 78 500 8 > "$O/probe_$spin.txt" 2>&1 || { tail -5 "$O/probe_$spin.txt"; exit 1; }
  python3 - "$O/t_$spin" "$spin" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "regwide" in r["Name"]:
            print(sys.argv[2], r["Name"][:48], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms")
PY
done
