set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for m in 0 4; do
  GSPARSE_CG_MODE=$m timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/b4.json 2>gpurun_out/b4.err || exit 1
  echo "mode $m: $(python -c "import json;d=json.load(open('gpurun_out/b4.json'));print(d['ms_per_step'], d['value'])")"
done
done
