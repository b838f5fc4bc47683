set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "all_cg_modes or blas_chunks" > gpurun_out/pytest_res.log 2>&1 || { tail -40 gpurun_out/pytest_res.log; exit 1; }
tail -3 gpurun_out/pytest_res.log
for cfg in "0 1 4" "4 1 4" "4 0 4" "4 1 8" "4 1 2"; do
  set -- $cfg
  GSPARSE_CG_MODE=$1 GSPARSE_RES_STOREQ=$2 GSPARSE_CG_RU=$3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 > gpurun_out/bench_m$1_$2_$3.json 2>gpurun_out/bench_m$1_$2_$3.err || exit 1
  echo "$cfg: $(python -c "import json;d=json.load(open('gpurun_out/bench_m$1_$2_$3.json'));print(d['ms_per_step'], d['kernels'])")"
done
