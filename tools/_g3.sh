set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "blas_chunks or column_blocks or all_cg_modes" > gpurun_out/pytest_res.log 2>&1 || { tail -30 gpurun_out/pytest_res.log; exit 1; }
tail -1 gpurun_out/pytest_res.log
for rep in 1 2; do
  GSPARSE_RES_PROF=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b3.json 2>gpurun_out/b3.err || exit 1
  echo "$rep $(grep resident gpurun_out/b3.err | tail -1) $(python -c "import json;d=json.load(open('gpurun_out/b3.json'));print(d['ms_per_step'])")"
done
