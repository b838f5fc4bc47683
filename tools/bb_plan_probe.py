"""GPU box: the staged backbone's plan stage (part 0 of N), host wall time and the
profile regions inside it (bb_plan_need / _fill / _cross), RMAT-18, Jaccard costs."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gnn-sparsification-research_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsparse import graphs  # noqa: E402
from gsparse._lib import Context  # noqa: E402
from gsparse.engine import Engine  # noqa: E402
from gsparse.metric_backbone import BackboneStages  # noqa: E402

ei = graphs.rmat(18, 8, seed=0)
n, E = 1 << 18, ei.shape[1]
dev = torch.device("cuda", 0)
ctx0 = Context(0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx0.set_graph_edge_index(n, src, dst)
sim = Engine(ctx0).jaccard()
p = sim / sim.max()
p[p <= 0] = p[p > 0].min() * 0.01
w = torch.from_numpy(np.ascontiguousarray((1.0 / p - 1.0)[:E])).to(dev)
ei_d = torch.stack([src, dst])
for N in (1, 8):
    ctx = Context(0)
    st = BackboneStages(ctx)
    for rep in range(3):
        st.begin(ei_d, n, w, 1e-9, 0, N)
        st.certify(0, N)
        torch.cuda.synchronize()
        ctx.profile(True)
        ctx.profile_reset()
        t0 = time.perf_counter()
        st.plan()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3
        prof = ctx.profile_read()
        ctx.profile(False)
        keep = torch.empty(E, dtype=torch.uint8, device=dev)
        st.finish(keep)
    print(json.dumps({"N": N, "plan_wall_ms": round(ms, 2),
                      "regions": {k: round(v["ms"], 3) for k, v in prof.items() if k.startswith("bb_plan")}}),
          flush=True)
