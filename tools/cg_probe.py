"""GPU box: time one ApproxER CG solve (gs_er_solve) on a Roman-like graph of n
nodes for `cols` JL columns, with the current GSPARSE_* environment (mode,
phase clock), e.g.  GSPARSE_CG_MODE=5 GSPARSE_RES_PROF=1 python tools/cg_probe.py 18000 256

usage: cg_probe.py N COLS [MAXITER] [BLAS_THREADS]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gnn-sparsification-research_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsparse import graphs  # noqa: E402
from gsparse._lib import Context  # noqa: E402
from gsparse.engine import Engine, jl_dim  # noqa: E402

n = int(sys.argv[1])
cols = int(sys.argv[2])
maxiter = int(sys.argv[3]) if len(sys.argv) > 3 else 500
bt = int(sys.argv[4]) if len(sys.argv) > 4 else 8
m = int(round(n * 32_927 / 22_662))
ei = graphs.roman_like(n, m, seed=0)
ctx = Context(0)
dev = torch.device("cuda", 0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx.set_graph_edge_index(n, src, dst)
eng = Engine(ctx)
k = max(cols, jl_dim(n, 0.3))
eng.er_prepare(k)
eng.er_project_device(np.random.default_rng(42), k)
eng.er_solve(0, cols, maxiter, 1e-6, bt)  # warm-up
ctx.synchronize()
t = time.perf_counter()
eng.er_solve(0, cols, maxiter, 1e-6, bt)
ctx.synchronize()
dt = time.perf_counter() - t
it = eng.er_iterations()[:cols]
print(f"n={n} cols={cols} iters_mean={it.mean():.1f} solve={dt*1e3:.2f} ms "
      f"per column-iteration per CU={dt / (it.sum() / min(cols, 256)) * 1e6:.2f} us", flush=True)
