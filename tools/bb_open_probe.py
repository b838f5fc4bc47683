"""GPU box: what the certificates leave open on RMAT-18 (Jaccard costs): after
gs_bb_begin + gs_bb_certify, the open columns' weights, and for the heaviest ones the
best landmark bound min_l D_l(u) + D_l(v) and the endpoints' degrees."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gnn-sparsification-research_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsparse import graphs  # noqa: E402
from gsparse._lib import Context  # noqa: E402
from gsparse.engine import Engine  # noqa: E402
from gsparse.metric_backbone import BackboneStages  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
ei = graphs.rmat(scale, 8, seed=0)
n = 1 << scale
E = ei.shape[1]
dev = torch.device("cuda", 0)
ctx0 = Context(0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx0.set_graph_edge_index(n, src, dst)
sim = Engine(ctx0).jaccard()
p = sim / sim.max()
p[p <= 0] = p[p > 0].min() * 0.01
cost = (1.0 / p - 1.0)[:E]
w = torch.from_numpy(np.ascontiguousarray(cost)).to(dev)
st = BackboneStages(Context(0))
K = st.begin(torch.stack([src, dst]), n, w, 1e-9, 0, 1)
D = torch.empty(K * n, dtype=torch.float64, device=dev)
C = torch.empty(K, dtype=torch.int32, device=dev)
st.landmarks_io(D, C, out=True)
st.certify(0, 1)
state = torch.empty(E, dtype=torch.uint8, device=dev)
st.state_io(state, out=True)
s = state.cpu().numpy()
D = D.cpu().numpy().reshape(n, K)
deg = np.bincount(ei[0], minlength=n)
big = cost.max()
out = {"E": int(E), "K": K, "complete": C.cpu().numpy().tolist(), "state_counts": np.bincount(s, minlength=4).tolist(),
       "max_cost": float(big), "cost_quantiles": np.quantile(cost, [0.1, 0.5, 0.9, 0.99]).tolist(),
       "n_maxcost_cols": int((cost == big).sum()), "open_maxcost": int(((cost == big) & (s == 0)).sum()),
       "open_weight_quantiles": np.quantile(cost[s == 0], [0.1, 0.5, 0.9, 0.99]).tolist() if (s == 0).any() else []}
deg = None
# the open columns' fate: finish the prune
nb = st.plan()
st.search(0, nb, 0, 1)
keep = torch.empty(E, dtype=torch.uint8, device=dev)
st.finish(keep)
k = keep.cpu().numpy().astype(bool)
op = s == 0
out["open"] = int(op.sum())
out["open_kept"] = int((op & k).sum())
out["open_pruned"] = int((op & ~k).sum())
out["open_kept_weight_q"] = np.quantile(cost[op & k], [0.1, 0.5, 0.9]).tolist() if (op & k).any() else []
out["open_pruned_weight_q"] = np.quantile(cost[op & ~k], [0.1, 0.5, 0.9]).tolist() if (op & ~k).any() else []
out["open_kept_maxcost"] = int((op & k & (cost == big)).sum())
out["open_pruned_maxcost"] = int((op & ~k & (cost == big)).sum())
out["batches"] = nb
print(json.dumps(out))
