"""Exact-ER timing probe: gs_exact_er on roman-like subgraphs of growing n,
fp64 MFMA GEMM rate from the context profiler (exact_er_dgemm entries carry
2 N^3 flops per launch)."""
import sys
import time

import numpy as np
import scipy.sparse as sp

sys.path.insert(0, "gnn-sparsification-research_amd")
from gsparse._lib import Context  # noqa: E402
from gsparse.engine import Engine  # noqa: E402
from gsparse import graphs  # noqa: E402

sizes = [int(a) for a in sys.argv[1:]] or [2000, 4096, 8192]
for n in sizes:
    rng = np.random.default_rng(n)
    m = 3 * n
    r = rng.integers(0, n, m)
    c = rng.integers(0, n, m)
    keep = r != c
    A = sp.coo_matrix((np.ones(keep.sum()), (r[keep], c[keep])), shape=(n, n)).tocsr()
    A = ((A + A.T) > 0).astype(np.float64).tocsr()
    ctx = Context(0)
    ctx.set_graph_csr(n, A.indptr, A.indices, A.data)
    eng = Engine(ctx)
    eng.exact_er()  # warm
    ctx.profile(True)
    ctx.profile_reset()
    t = time.time()
    er = eng.exact_er()
    dt = time.time() - t
    prof = ctx.profile_read()
    ctx.profile(False)
    g = prof.get("exact_er_dgemm", {"launches": 0, "ms": 0, "bytes": 0})
    tf = g["bytes"] / (g["ms"] * 1e-3) / 1e12 if g["ms"] else 0
    print(f"n={n} nnz={A.nnz} iters={eng.exact_er_iterations} total={dt*1e3:.1f} ms "
          f"gemm launches={g['launches']} gemm_ms={g['ms']:.1f} per={g['ms']/max(g['launches'],1):.3f} "
          f"fp64 {tf:.1f} TFLOP/s  er[:3]={er[:3]}", flush=True)
