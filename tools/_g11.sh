set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "exact_er" > gpurun_out/pytest_xer.log 2>&1 || { grep -E "Error|assert|Mismatch|Max" gpurun_out/pytest_xer.log | head -20; tail -3 gpurun_out/pytest_xer.log; exit 1; }
tail -1 gpurun_out/pytest_xer.log
GSPARSE_XER_PANEL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "exact_er_device or components" > gpurun_out/pytest_xer1.log 2>&1 || { tail -3 gpurun_out/pytest_xer1.log; exit 1; }
tail -1 gpurun_out/pytest_xer1.log
for P in 8; do
GSPARSE_XER_PANEL=$P timeout -k 10 200 python bench.py --workload exact_er --xer-n 22662 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bxer.json 2>gpurun_out/bxer.err || { tail -3 gpurun_out/bxer.err; exit 1; }
echo "P=$P roman $(python -c "import json;d=json.load(open('gpurun_out/bxer.json'));print(d['ms_per_step'], d['roofline']['achieved'])")"
done
timeout -k 10 120 python bench.py --workload exact_er --no-cpu-baseline > gpurun_out/bxer.json 2>gpurun_out/bxer.err || exit 1
echo "cora $(python -c "import json;d=json.load(open('gpurun_out/bxer.json'));print(d['ms_per_step'], d['roofline']['achieved'])")"
