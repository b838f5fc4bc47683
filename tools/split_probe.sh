#!/bin/bash
# GPU box: the split last round of the register-resident CG.  For the tail column
# counts of a rank at N = 2 / 4 / 8 (57, 157, 78 Roman columns), the solve time with
# the split form forced to P parts vs automatic vs off.  usage: split_probe.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-split}
mkdir -p "$O"
for c in 78 57 157; do
  for p in auto 0 2 3 4 8; do
    if [ "$p" = auto ]; then env=""; else env="GSPARSE_REG_SPLIT=$p"; fi
    env $env timeout -k 10 200 python tools/cg_probe.py 22662 $c 500 8 > "$O/c${c}_p$p.txt" 2>&1 || { tail -5 "$O/c${c}_p$p.txt"; exit 1; }
    echo "cols=$c split=$p $(grep solve= $O/c${c}_p$p.txt)"
  done
done
