#!/bin/bash
# round 6: the select with 2-bit keep codes and async library calls: the distributed
# tests, the per-rank probe, the N = 2 / 8 rehearsals of the R-MAT line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06w
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > "$O/dist.log" 2>&1 || { tail -40 "$O/dist.log"; exit 1; }
tail -1 "$O/dist.log"
timeout -k 10 500 python -u tools/jsel_probe.py 22 0.5 3 > "$O/jsel_probe.jsonl" 2> "$O/jsel_probe.err" || { tail -20 "$O/jsel_probe.err"; exit 1; }
tail -1 "$O/jsel_probe.jsonl" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:(v['max_device_ms'],v['max_wall_ms'],v['mask_equals_one_gpu_topk'],v['part0_kernels_ms']) for k,v in d['per_n'].items()})"
for N in 2 8; do
  GSPARSE_REHEARSE=1 timeout -k 10 400 python bench.py --gpus $N --workload rmat --steps 3 --warmup 1 --no-cpu-baseline > "$O/rmat_n$N.json" 2> "$O/rmat_n$N.err" || { tail -20 "$O/rmat_n$N.err"; exit 1; }
  grep '^{' "$O/rmat_n$N.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('rmat N=$N rehearsal', d['ms_per_step'], d['rank_ms_per_step'], d['config']['topk'])"
done
