set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "all_cg_modes or blas_chunks or column_blocks" 2>&1 | tail -3 || exit 1
for n in 12000 18000 22662; do
  echo "== wide n=$n"; GSPARSE_CG_MODE=5 GSPARSE_RES_PROF=1 timeout -k 10 120 python tools/cg_probe.py $n 256 500 8 2>&1 | grep -v amdgpu.ids || exit 1
done
echo "== narrow 22662"; GSPARSE_REG_NT=256 GSPARSE_CG_MODE=5 GSPARSE_RES_PROF=1 timeout -k 10 120 python tools/cg_probe.py 22662 256 500 8 2>&1 | grep -v amdgpu.ids || exit 1
echo "== mode4 22662"; GSPARSE_CG_MODE=4 GSPARSE_RES_PROF=1 timeout -k 10 120 python tools/cg_probe.py 22662 256 500 8 2>&1 | grep -v amdgpu.ids || exit 1
