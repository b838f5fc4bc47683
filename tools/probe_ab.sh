#!/bin/bash
# GPU box: CG probe (Roman size, 256 columns x 500 iterations, phase clock) for each
# GSPARSE_* setting given as an argument ("-" = defaults), e.g.
#   probe_ab.sh TAG - GSPARSE_REG_QR=0
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1
shift
mkdir -p "$O"
i=0
for cfg in "$@"; do
  i=$((i+1))
  envs=(); [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  env "${envs[@]}" GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$O/probe_$i.txt" 2>&1 || { tail -20 "$O/probe_$i.txt"; exit 1; }
  echo "[$cfg]"; grep -v "^\s*$" "$O/probe_$i.txt" | tail -2
done
