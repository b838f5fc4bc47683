#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05splitwr
mkdir -p "$O"
PKG=gnn-sparsification-research_amd/gsparse
for rep in 1 2; do
for v in main nopub noxst nowr; do
  if [ "$v" = main ]; then lib=$PWD/$PKG/libgsparse.so; else lib=$PWD/$PKG/libgsparse_$v.so; fi
  for c in 114 78; do
    GSPARSE_LIB=$lib timeout -k 10 200 python tools/cg_probe.py 22662 $c 500 8 > "$O/${v}_c${c}_$rep.txt" 2>&1 || { tail -5 "$O/${v}_c${c}_$rep.txt"; exit 1; }
    echo "$v cols=$c $(grep solve= $O/${v}_c${c}_$rep.txt)"
  done
done
done
