#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R06A_TAG=r06g bash tools/r06a_check.sh || exit 1
bash tools/r06f_jac_ab.sh
# the split tail (2 parts per column) vs whole columns, now that whole columns are faster
for rep in 1; do
  for sp in default 0; do
    if [ $sp = default ]; then envs=""; else envs="GSPARSE_REG_SPLIT=0"; fi
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --box-order-steps 0 > gpurun_out/r06f/roman_split_${sp}_$rep.json 2> gpurun_out/r06f/roman_split_${sp}_$rep.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/r06f/roman_split_${sp}_$rep.json'));print('split=$sp rep $rep ms/step',d['ms_per_step'])"
  done
done
# whole columns with x in Xc and q stored (GS_CG_XG) vs x in registers
bash tools/variant_ab.sh r06g2 main xg
