#!/bin/bash
# GPU box (one GPU): the N = 2 bench path rehearsed with two ranks sharing the card
# (gloo); the split CG's hand-offs may give up while the other rank holds CUs, and
# the tail is then re-solved whole -- this checks that the path completes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-n2}
mkdir -p "$O"
GSPARSE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline \
    > "$O/bench_n2.json" 2> "$O/bench_n2.err" || { tail -20 "$O/bench_n2.err"; exit 1; }
grep -c "timed out" "$O/bench_n2.err" || true
grep '^{' "$O/bench_n2.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('N=2 rehearsal ms/step', d['ms_per_step'], 'value', d['value'])"
