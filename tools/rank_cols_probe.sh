#!/bin/bash
# GPU box: one rank's share of the Roman JL columns at N = 2, 4, 8 (1337, 669, 334
# columns, 500 CG iterations), solved with and without the split last round.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-rankcols}
mkdir -p "$O"
for cols in 334 669 1337; do
  for sp in auto 0; do
    if [ $sp = auto ]; then unset GSPARSE_REG_SPLIT; else export GSPARSE_REG_SPLIT=0; fi
    timeout -k 10 200 python tools/cg_probe.py 22662 $cols > "$O/c${cols}_$sp.txt" 2>&1 || { tail -20 "$O/c${cols}_$sp.txt"; exit 1; }
    echo "cols=$cols split=$sp: $(grep solve= "$O/c${cols}_$sp.txt")"
  done
done
