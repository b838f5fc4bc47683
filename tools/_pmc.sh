set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc4}
mkdir -p $O
i=0
for set in "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_IFETCH SQ_LDS_ADDR_CONFLICT"; do
  i=$((i+1))
  GSPARSE_CG_MODE=5 timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/cg_probe.py 22662 256 100 8 > $O/p$i.log 2>&1 || { echo "pass failed: $set"; exit 1; }
done
python3 tools/pmc_summary.py $O/summary.json $O/p1 $O/p2 | grep regwide
