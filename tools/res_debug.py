"""Resident CG (mode 4) probe: tiny graphs, increasing maxiter, timed."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "gnn-sparsification-research_amd"), os.path.join(ROOT, "oracle")]
os.environ.setdefault("GSPARSE_CG_MODE", "4")
import numpy as np, torch
import gsparse, gsparse_oracle as O
from gsparse import graphs
name = sys.argv[1] if len(sys.argv) > 1 else "path"
if name == "path":
    n = 6
    ei = np.array([[0, 1, 2, 3, 4], [1, 2, 3, 4, 5]]); ei = np.concatenate([ei, ei[::-1]], 1)
else:
    n = 2000
    ei = graphs.roman_like(n, 2900, seed=1)
ip, ix, d = O.canonical_csr(ei, n)
sp_ = gsparse.GraphSparsifier(gsparse.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
for it in [1, 2, 5, 50]:
    t0 = time.time()
    er = sp_._engine.approx_er(epsilon=2.0, max_cg_iters=it, blas_threads=1)
    ref = O.approx_er(ip, ix, d, n, epsilon=2.0, max_cg_iters=it, impl="c", blas_threads=1)
    print(name, it, round(time.time() - t0, 3), "equal" if np.array_equal(er.view(np.uint64), ref.view(np.uint64)) else f"DIFF {np.max(np.abs(er-ref))}", flush=True)
