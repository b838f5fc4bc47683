"""Time the CG solve on a column block of the Roman workload (what one rank
of an N-GPU run solves): k/N columns."""
import sys, time, json
import numpy as np, torch
sys.path.insert(0, 'gnn-sparsification-research_amd')
from gsparse import graphs
from gsparse._lib import Context
from gsparse.engine import Engine, jl_dim, er_split

ei, n = graphs.roman_like(), 22662
ctx = Context(0)
ctx.set_graph_edge_index(n, torch.from_numpy(ei[0].copy()).cuda(), torch.from_numpy(ei[1].copy()).cuda())
eng = Engine(ctx)
k = jl_dim(n, 0.3)
eng.er_prepare(k)
eng.er_project_device(np.random.default_rng(42), k)
for parts in [1, 2, 4, 8]:
    b = er_split(k, parts) if parts > 1 else [0, k]
    c0, c1 = b[0], b[1]
    eng.er_solve(c0, c1, 500, 1e-6, 8)  # warm
    torch.cuda.synchronize()
    ctx.profile(True); ctx.profile_reset()
    t = time.perf_counter()
    eng.er_solve(c0, c1, 500, 1e-6, 8)
    eng.er_scores(c0, c1, finalize=False)
    dt = time.perf_counter() - t
    prof = ctx.profile_read(); ctx.profile(False)
    print(json.dumps({"parts": parts, "cols": c1 - c0, "s": round(dt, 4),
                      "kernels": {kk: round(v["ms"], 2) for kk, v in prof.items()}}), flush=True)
