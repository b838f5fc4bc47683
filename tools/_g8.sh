set -o pipefail
mkdir -p gpurun_out
for sl in 256 128 64 32; do
  GSPARSE_CG_SLOTS=$sl GSPARSE_RES_PROF=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/b8.json 2>gpurun_out/b8.err || exit 1
  echo "slots=$sl $(grep resident gpurun_out/b8.err | tail -1) $(python -c "import json;d=json.load(open('gpurun_out/b8.json'));print(d['ms_per_step'])")"
done
