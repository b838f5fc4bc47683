#!/bin/bash
# round 6: the split last round against whole columns, per rank share of the Roman JL
# columns (N = 1 / 2 / 4 / 8: 2674 / 1337 / 669 / 334 columns)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06x
mkdir -p "$O"
for cols in 334 669 1337 2674; do
  for sp in auto 0; do
    if [ $sp = auto ]; then unset GSPARSE_REG_SPLIT; else export GSPARSE_REG_SPLIT=0; fi
    timeout -k 10 200 python tools/cg_probe.py 22662 $cols > "$O/c${cols}_$sp.txt" 2>&1 || { tail -20 "$O/c${cols}_$sp.txt"; exit 1; }
    echo "cols=$cols split=$sp: $(grep solve= "$O/c${cols}_$sp.txt")"
  done
done
