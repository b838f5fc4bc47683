#!/bin/bash
# GPU box: Roman-size CG probe (256 columns x 500 iterations, phase clock) for each
# library build given (NAME -> gnn-sparsification-research_amd/gsparse/libgsparse_NAME.so,
# "main" = libgsparse.so); NAME+ also runs the mode-5 parity subset on it first.
# usage: probe_libs.sh TAG NAME...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; shift
mkdir -p "$O"
PKG=gnn-sparsification-research_amd/gsparse
for v in "$@"; do
  par=0; case $v in *+) par=1; v=${v%+} ;; esac
  if [ "$v" = main ]; then lib=$PWD/$PKG/libgsparse.so; else lib=$PWD/$PKG/libgsparse_$v.so; fi
  if [ $par = 1 ]; then
    GSPARSE_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
        -k "all_cg_modes or blas_chunks or column_blocks or roman_full" > "$O/pytest_$v.log" 2>&1 || { tail -30 "$O/pytest_$v.log"; exit 1; }
    echo "$v: $(tail -1 $O/pytest_$v.log)"
  fi
  GSPARSE_LIB=$lib GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$O/probe_$v.txt" 2>&1 || { tail -20 "$O/probe_$v.txt"; exit 1; }
  echo "[$v] $(grep -v '^\s*$' $O/probe_$v.txt | tail -2 | tr '\n' ' ')"
done
