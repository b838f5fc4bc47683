#!/bin/bash
# GPU box: register-resident CG (mode 5) parity tests, then the default line with the phase clock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-m5}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread \
    -k "all_cg_modes or blas_chunks or column_blocks" > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
GSPARSE_RES_PROF=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench5.json" 2> "$O/bench5.err" || { tail -20 "$O/bench5.err"; exit 1; }
grep "resident" "$O/bench5.err" | tail -2; cat "$O/bench5.json"
GSPARSE_CG_MODE=4 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$O/bench4.json" 2> "$O/bench4.err" || { tail -20 "$O/bench4.err"; exit 1; }
python3 -c "import json;a=json.load(open('$O/bench5.json'));b=json.load(open('$O/bench4.json'));print('mode5 ms/step',a['ms_per_step'],'mode4',b['ms_per_step'])"
