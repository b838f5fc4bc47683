set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_default.json
bash tools/profile_bench.sh gpurun_out/prof_roman > gpurun_out/prof_roman.log 2>&1 || { tail -5 gpurun_out/prof_roman.log; exit 1; }
tail -3 gpurun_out/prof_roman.log
