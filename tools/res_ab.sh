#!/bin/bash
# GPU box: A/B of resident-solver env variants on the default line (phase clock + step time).
# usage: res_ab.sh "ENV=V ..." "ENV=V ..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg GSPARSE_RES_PROF=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/b3.json 2>gpurun_out/b3.err || exit 1
  echo "[$cfg] $(grep -i resident gpurun_out/b3.err | tail -1 | cut -c40-) $(python -c "import json;d=json.load(open('gpurun_out/b3.json'));print(d['ms_per_step'])")"
done
