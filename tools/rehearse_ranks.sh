#!/bin/bash
# GPU box (one GPU): the N-rank bench paths rehearsed with N ranks sharing the card
# (GSPARSE_REHEARSE=1: gloo, split CG off), each workload; then --gpus 2 without the
# rehearsal flag must refuse (one GPU visible).  usage: rehearse_ranks.sh TAG [N]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-ranks}; N=${2:-2}
mkdir -p "$O"
for w in roman rmat backbone; do
  extra=""; [ $w = backbone ] && extra="--bb-graph roman"
  GSPARSE_REHEARSE=1 timeout -k 10 300 python bench.py --gpus $N --workload $w $extra --steps 2 --warmup 1 --no-cpu-baseline \
      > "$O/${w}_n$N.json" 2> "$O/${w}_n$N.err" || { tail -20 "$O/${w}_n$N.err"; exit 1; }
  grep '^{' "$O/${w}_n$N.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$w N=$N rehearsal', d['n_gpus'], 'ranks', d['ms_per_step'], 'ms/step', d['config'].get('parallelism'))"
done
if timeout -k 10 120 python bench.py --gpus 2 --steps 1 --warmup 0 --no-cpu-baseline > "$O/refuse.out" 2>&1; then
  echo "--gpus 2 on one GPU did not refuse"; exit 1
fi
tail -1 "$O/refuse.out"
