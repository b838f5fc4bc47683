"""Time the device normal stream + projection of the Roman ApproxER (3 calls)."""
import sys, time
import numpy as np, torch
sys.path.insert(0, 'gnn-sparsification-research_amd')
from gsparse import graphs
from gsparse._lib import Context
from gsparse.engine import Engine, jl_dim

ei, n = graphs.roman_like(), 22662
ctx = Context(0)
ctx.set_graph_edge_index(n, torch.from_numpy(ei[0].copy()).cuda(), torch.from_numpy(ei[1].copy()).cuda())
eng = Engine(ctx)
k = jl_dim(n, 0.3)
for i in range(3):
    eng.er_prepare(k)
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.er_project_device(np.random.default_rng(42), k)
    torch.cuda.synchronize()
    print("project_device s", round(time.perf_counter() - t, 4), flush=True)
