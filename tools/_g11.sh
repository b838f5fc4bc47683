set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "exact_er" > gpurun_out/pytest_xer.log 2>&1 || { grep -E "Error|assert|Mismatch|Max" gpurun_out/pytest_xer.log | head -20; tail -3 gpurun_out/pytest_xer.log; exit 1; }
tail -1 gpurun_out/pytest_xer.log
for m in chol ns; do
GSPARSE_XER_METHOD=$m timeout -k 10 120 python bench.py --workload exact_er --no-cpu-baseline > gpurun_out/bxer.json 2>gpurun_out/bxer.err || { tail -3 gpurun_out/bxer.err; exit 1; }
echo "$m cora $(python -c "import json;d=json.load(open('gpurun_out/bxer.json'));print(d['ms_per_step'], d['roofline']['achieved'])")"
done
GSPARSE_XER_METHOD=chol timeout -k 10 200 python bench.py --workload exact_er --xer-n 22662 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bxer.json 2>gpurun_out/bxer.err || { tail -3 gpurun_out/bxer.err; exit 1; }
echo "chol roman $(python -c "import json;d=json.load(open('gpurun_out/bxer.json'));print(d['ms_per_step'], d['roofline']['achieved'])")"
