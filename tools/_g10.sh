set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --workload backbone --bb-graph roman > gpurun_out/bench_bb_roman.json 2> gpurun_out/bench_bb_roman.err || exit 1
timeout -k 10 400 python bench.py --workload backbone --steps 1 > gpurun_out/bench_bb_rmat.json 2> gpurun_out/bench_bb_rmat.err || exit 1
cat gpurun_out/bench_bb_rmat.json
bash tools/profile_bench.sh gpurun_out/prof_backbone --workload backbone > gpurun_out/prof_bb.log 2>&1 || { tail -5 gpurun_out/prof_bb.log; exit 1; }
echo profiled
