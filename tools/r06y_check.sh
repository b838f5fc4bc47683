#!/bin/bash
# round 6: one rank's Jaccard-T work with the distributed select (tools/jsel_probe.py),
# the N-rank bench paths rehearsed on the one GPU, and the split-tail A/B repeated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06y
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_pins.py -x -v --timeout 400 --timeout-method thread -k roman > "$O/pins_roman.log" 2>&1 || { tail -30 "$O/pins_roman.log"; exit 1; }
tail -1 "$O/pins_roman.log"
timeout -k 10 500 python -u tools/jsel_probe.py 22 0.5 3 > "$O/jsel_probe.jsonl" 2> "$O/jsel_probe.err" || { tail -20 "$O/jsel_probe.err"; exit 1; }
tail -1 "$O/jsel_probe.jsonl" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k:(v['max_device_ms'],v['max_wall_ms'],v['mask_equals_one_gpu_topk']) for k,v in d['per_n'].items()}, 'replicated topk', d['replicated_topk_ms'])"
bash tools/rehearse_ranks.sh r06y_ranks 2 || exit 1
GSPARSE_REHEARSE=1 timeout -k 10 400 python bench.py --gpus 8 --workload rmat --steps 2 --warmup 1 --no-cpu-baseline > "$O/rmat_n8.json" 2> "$O/rmat_n8.err" || { tail -20 "$O/rmat_n8.err"; exit 1; }
grep '^{' "$O/rmat_n8.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('rmat N=8 rehearsal', d['ms_per_step'], d['config']['parallelism'], d['config']['topk'])"
for rep in 1 2 3; do
  for sp in default 0; do
    if [ $sp = default ]; then envs=""; else envs="GSPARSE_REG_SPLIT=0"; fi
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --box-order-steps 0 > "$O/roman_split_${sp}_$rep.json" 2> "$O/roman_split_${sp}_$rep.err" || exit 1
    python3 -c "import json;d=json.load(open('$O/roman_split_${sp}_$rep.json'));print('split=$sp rep $rep ms/step',d['ms_per_step'])"
  done
done
# the secondary bench lines again, now joined to this tree's committed PMC summaries
for wl in roman rmat backbone arxiv; do
  timeout -k 10 400 python bench.py --workload $wl --steps 5 --warmup 2 > "$O/bench_$wl.json" 2> "$O/bench_$wl.err" || { tail -5 "$O/bench_$wl.err"; exit 1; }
  python3 -c "import json;a=json.load(open('$O/bench_$wl.json'));r=a['roofline'];print('$wl ms/step',a['ms_per_step'],'frac',r.get('frac'),'traffic',r.get('traffic'))"
done
