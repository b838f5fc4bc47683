"""Debug helper: GPU ApproxER vs the C oracle at increasing maxiter."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-sparsification-research_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import gsparse_oracle as O
from gsparse._lib import Context
from gsparse.engine import Engine, jl_dim
for name in sys.argv[1:]:
    z = np.load(os.path.join(ROOT, "tests/golden", name + ".npz"))
    n = int(z["num_nodes"]); ip, ix, d = z["indptr"], z["indices"], z["data"]
    ctx = Context(0); ctx.set_graph_csr(n, ip, ix, d); e = Engine(ctx)
    k = jl_dim(n, 0.3)
    Y, m, kk = O.approx_er_projection(ip, ix, n)
    L = O.laplacian_reg(ip, ix, d, n)
    rows = O.csr_rows(ip)
    for mi in [1, 2, 3, 500]:
        e.er_prepare(k); e.er_project_host(np.random.default_rng(42), k)
        e.er_solve(0, k, mi, 1e-6, 1)
        g = e.er_scores(0, k, True)
        its_g = e.er_iterations()
        Z, its = O.cg(L, Y, mi, 1e-6, 1)
        ref = O.er_from_z(ip, ix, Z)
        bad = np.nonzero(g != ref)[0]
        print(name, n, mi, "mismatch edges", len(bad), "iters equal", np.array_equal(its_g, its), flush=True)
        if len(bad):
            badc = []
            for c in range(0, k):
                gc = e.er_scores(c, c + 1, False)
                rc = (Z[rows, c] - Z[ix, c]) ** 2
                if not np.array_equal(gc, rc):
                    badc.append(c)
            print("  bad columns", len(badc), badc[:20])
            c = badc[0]
            gc = e.er_scores(c, c + 1, False); rc = (Z[rows, c] - Z[ix, c]) ** 2
            bb = np.nonzero(gc != rc)[0]
            print("  col", c, "bad edges", len(bb), "first", bb[:10], "rows", rows[bb[:10]], ix[bb[:10]])
            print("  rel", np.max(np.abs(gc-rc)/np.maximum(np.abs(rc),1e-300)))
            break
