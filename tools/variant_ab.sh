#!/bin/bash
# GPU box: A/B of libgsparse builds.  For each variant V (libgsparse_V.so, made by
# `make -C gnn-sparsification-research_amd/csrc variant V=... VFLAGS=...`; "main" =
# the default libgsparse.so): the mode-5 parity subset, then the Roman-size CG probe
# (per column-iteration) and the default bench line.  usage: variant_ab.sh TAG V...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; shift
O=gpurun_out/$T
mkdir -p "$O"
PKG=gnn-sparsification-research_amd/gsparse
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/$PKG/libgsparse.so; else lib=$PWD/$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "all_cg_modes or blas_chunks or column_blocks or roman_full" > "$O/pytest_$v.log" 2>&1 || { tail -30 "$O/pytest_$v.log"; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  GSPARSE_LIB=$lib GSPARSE_RES_PROF=1 timeout -k 10 200 python tools/cg_probe.py 22662 256 > "$O/probe_$v.txt" 2>&1 || { tail -20 "$O/probe_$v.txt"; exit 1; }
  grep -v "^\s*$" "$O/probe_$v.txt" | tail -2
  GSPARSE_LIB=$lib timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$O/bench_$v.json" 2> "$O/bench_$v.err" || { tail -20 "$O/bench_$v.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$O/bench_$v.json'));print('$v ms/step',a['ms_per_step'],'kernel ms',a['roofline']['avg_launch_ms'])"
done
