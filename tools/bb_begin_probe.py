"""GPU box: the staged backbone's begin stage (graph build + landmark searches) of part
0 of N, per profile region, for both landmark forms (GSPARSE_BB_LMCOOP) and some
workgroup counts (GSPARSE_BB_LMW).  usage: bb_begin_probe.py [SCALE]"""
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

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
ei = graphs.rmat(scale, 8, seed=0)
n = 1 << scale
dev = torch.device("cuda", 0)
ctx0 = Context(0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx0.set_graph_edge_index(n, src, dst)
sim = Engine(ctx0).jaccard()
p = sim / sim.max()
p[p <= 0] = p[p > 0].min() * 0.01
w = torch.from_numpy(np.ascontiguousarray((1.0 / p - 1.0)[:ei.shape[1]])).to(dev)
ei_d = torch.stack([src, dst])
os.environ["GSPARSE_BB_DEBUG"] = "1"
for cfg in (("0", "0"), ("1", "0"), ("1", "4"), ("1", "16"), ("1", "64")):
    os.environ["GSPARSE_BB_LMCOOP"], lmw = cfg
    if lmw != "0":
        os.environ["GSPARSE_BB_LMW"] = lmw
    else:
        os.environ.pop("GSPARSE_BB_LMW", None)
    for N in (1, 8):
        ctx = Context(0)
        st = BackboneStages(ctx)
        for rep in range(2):
            ctx.profile(True)
            ctx.profile_reset()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st.begin(ei_d, n, w, 1e-9, 0, N)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3
            prof = ctx.profile_read()
        print(json.dumps({"lmcoop": cfg[0], "lmw": lmw, "N": N, "begin_ms": round(ms, 2),
                          "regions": {k: v for k, v in prof.items() if k.startswith("bb_")}}), flush=True)
