import sys, time, numpy as np, torch
sys.path.insert(0, 'gnn-sparsification-research_amd')
from gsparse import graphs
from gsparse.metric_backbone import backbone_mask
from gsparse._lib import Context
from gsparse.engine import Engine
for name, (ei, n) in [("roman", (graphs.roman_like(), 22662)), ("rmat16", (graphs.rmat(16, 8, seed=0), 1 << 16)), ("rmat18", (graphs.rmat(18, 8, seed=0), 1 << 18))]:
    ctx = Context(0)
    ctx.set_graph_edge_index(n, torch.from_numpy(ei[0].copy()).cuda(), torch.from_numpy(ei[1].copy()).cuda())
    eng = Engine(ctx)
    jac = eng.jaccard()
    # cost aligned to edge_index columns: scores are CSR order -> use reference rule via GraphSparsifier
    import gsparse
    d = gsparse.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp = gsparse.GraphSparsifier(d, "cpu")
    s = sp.compute_scores("jaccard")
    cost = sp._scores_to_cost(s, "jaccard")
    t = time.time()
    mask, nr = backbone_mask(ei, n, cost, ctx=ctx, return_relax=True)
    dt = time.time() - t
    print(name, "E", ei.shape[1], "kept", int(mask.sum()), "relax", nr, "s", round(dt, 3), flush=True)
