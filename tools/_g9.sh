set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "backbone" > gpurun_out/pytest_bb.log 2>&1 || { tail -30 gpurun_out/pytest_bb.log; exit 1; }
tail -1 gpurun_out/pytest_bb.log
for rl in auto 0; do
env $( [ $rl = auto ] || echo GSPARSE_BB_RELABEL=$rl ) timeout -k 10 300 python bench.py --workload backbone --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/bench_bb_rmat.json 2> gpurun_out/bench_bb_rmat.err || exit 1
echo "relabel=$rl $(python -c "import json;d=json.load(open('gpurun_out/bench_bb_rmat.json'));print(d['ms_per_step'], d['config']['kept'], d['roofline']['relaxations_per_launch_rank0'])")"
done
timeout -k 10 300 python bench.py --workload backbone --bb-graph roman --no-cpu-baseline > gpurun_out/bench_bb_roman.json 2> gpurun_out/bench_bb_roman.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bench_bb_roman.json'));print('roman', d['ms_per_step'], d['config']['kept'])"
