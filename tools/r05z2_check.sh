#!/bin/bash
# GPU box: Jaccard home-bucket branch-free probe (main) vs the per-element search loop (jfp0):
# the R-MAT-22 pin, the RMAT step time (A/B/A/B), and each build's FETCH_SIZE.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05z2
mkdir -p "$O"
PKG=$PWD/gnn-sparsification-research_amd/gsparse
timeout -k 10 600 python -u -m pytest tests/test_gpu_rmat22.py tests/test_gpu_parity.py -m gpu -x -q --timeout 500 --timeout-method thread \
    -k "rmat22 or jaccard or common" > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
for rep in 1 2; do
  for v in main jfp0; do
    if [ "$v" = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
    GSPARSE_LIB=$lib timeout -k 10 300 python bench.py --workload rmat --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_${v}_$rep.json" 2> "$O/bench_${v}_$rep.err" || { tail -5 "$O/bench_${v}_$rep.err"; exit 1; }
    python3 -c "import json;a=json.load(open('$O/bench_${v}_$rep.json'));print('$v', a['ms_per_step'], a['roofline']['avg_launch_ms'])"
  done
done
for v in main jfp0; do
  if [ "$v" = main ]; then lib=$PKG/libgsparse.so; else lib=$PKG/libgsparse_$v.so; fi
  GSPARSE_LIB=$lib timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fetch_$v" -o run -- \
      python3 bench.py --workload rmat --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline > "$O/pmc_$v.json" 2> "$O/pmc_$v.err" || { tail -5 "$O/pmc_$v.err"; exit 1; }
  GSPARSE_LIB=$lib timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/write_$v" -o run -- \
      python3 bench.py --workload rmat --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline > "$O/pmcw_$v.json" 2> "$O/pmcw_$v.err" || { tail -5 "$O/pmcw_$v.err"; exit 1; }
  python3 tools/pmc_summary.py --calls=1 "$O/pmc_summary_$v.json" "$O/fetch_$v" "$O/write_$v" > "$O/pmc_summary_$v.txt"
  python3 - "$O/pmc_summary_$v.json" "$v" <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
tot = 0.0
for k, v in d.items():
    if k.startswith("_") or "jac" not in k:
        continue
    tot += (2 * v.get("FETCH_SIZE_KB_per_launch", 0) + v.get("WRITE_SIZE_KB_per_launch", 0)) * v["launches"]
print(sys.argv[2], "jaccard kernels 2F+W GB per call:", round(tot / 1e6, 2))
EOF
done
echo done
