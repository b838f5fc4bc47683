set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "column_blocks or blas_chunks" > gpurun_out/pytest_res.log 2>&1 || { tail -30 gpurun_out/pytest_res.log; exit 1; }
tail -1 gpurun_out/pytest_res.log
timeout -k 10 300 python bench.py --workload rmat --no-cpu-baseline > gpurun_out/bench_rmat.json 2> gpurun_out/bench_rmat.err || exit 1
cat gpurun_out/bench_rmat.json
bash tools/profile_bench.sh gpurun_out/prof_arxiv --workload arxiv > gpurun_out/prof_arxiv.log 2>&1 || { tail -5 gpurun_out/prof_arxiv.log; exit 1; }
cat gpurun_out/prof_arxiv/bench_trace.json
