#!/bin/bash
# GPU box: RMAT-18 backbone step time per env configuration.
# usage: bb_ab.sh "ENV=V ..." "ENV=V ..." ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --workload backbone ${BB_ARGS:---steps 1} --warmup 1 --no-cpu-baseline > gpurun_out/bbm.json 2>gpurun_out/bbm.err || { tail -5 gpurun_out/bbm.err; exit 1; }
  echo "[$cfg] $(python -c "import json;d=json.load(open('gpurun_out/bbm.json'));print(d['ms_per_step'], d['config']['kept'])")"
done
