#!/bin/bash
# rocprofv3 summaries of a bench workload (run on the GPU box).
# Pass 1: kernel trace + stats; passes 2/3: HBM bytes (FETCH_SIZE, WRITE_SIZE)
# in separate runs (MI355X_MICROARCH.md: TCC slots; FETCH_SIZE reads 1/2 of
# the bytes of a wide coalesced stream on gfx950); pass 4: L2 hit/miss; pass 5:
# SQ issue and wait counters.  The summary carries the sources' hash
# (tools/provenance.py), which bench.py checks before using it.
# usage: profile_bench.sh OUTDIR [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
shift || true
ARGS="$*"
mkdir -p "$OUT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --box-order-steps 0 --no-cpu-baseline $ARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || exit $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline $ARGS > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err" || exit $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline $ARGS > "$OUT/bench_write.json" 2> "$OUT/write.err" || exit $?
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/l2" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline $ARGS > "$OUT/bench_l2.json" 2> "$OUT/l2.err" || exit $?
# (the counter passes run exactly one call of each region: --steps 1 --warmup 0, no
# box-order re-run, so the summary's --calls=1 divides by the right count)
# pass 5: SQ issue / wait counters (bench.py's on_chip fields)
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_BRANCH --output-format csv -d "$OUT/sq" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --box-order-steps 0 --no-cpu-baseline $ARGS > "$OUT/bench_sq.json" 2> "$OUT/sq.err" || exit $?
python3 tools/pmc_summary.py --calls=1 "$OUT/pmc_summary.json" "$OUT/fetch" "$OUT/write" "$OUT/l2" "$OUT/sq" > "$OUT/pmc_summary.txt"
echo "profile done"
