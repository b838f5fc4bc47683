"""GPU box: per-batch timeline of the backbone's pair certificate (GSPARSE_BB_TRACE on
gs_bb_certify's PAIR launch), RMAT-18, Jaccard costs: duration vs radius / relaxations."""
import json
import os
import sys
import tempfile

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
st = BackboneStages(Context(0))
path = os.path.join(os.environ.get("BB_TRACE_DIR", tempfile.gettempdir()), "pair_trace.jsonl")
if os.path.exists(path):
    os.remove(path)
st.begin(torch.stack([src, dst]), n, w, 1e-9, 0, 1)
os.environ["GSPARSE_BB_TRACE"] = path
st.certify(0, 1)
os.environ.pop("GSPARSE_BB_TRACE")
keep = torch.empty(E, dtype=torch.uint8, device=dev)
st.plan()
st.finish(keep)
d = json.loads(open(path).readline())
rec = np.array(d["rec"], dtype=np.float64)
t0 = (rec[:, 0] - rec[:, 0].min()) / 1e5
t1 = (rec[:, 1] - rec[:, 0].min()) / 1e5
dur, rad, rel = t1 - t0, rec[:, 3], rec[:, 5]
print(json.dumps({"pairs": len(rec), "span_ms": round(float(t1.max()), 1), "mean_ms": round(float(dur.mean()), 3),
                  "dur_q": np.quantile(dur, [0.5, 0.9, 0.99, 1.0]).round(2).tolist(),
                  "radius_q": np.quantile(rad, [0.1, 0.5, 0.9, 0.99, 1.0]).round(1).tolist(),
                  "relax_q": np.quantile(rel, [0.5, 0.9, 0.99, 1.0]).tolist(), "relax_sum": float(rel.sum()),
                  "corr_dur_relax": round(float(np.corrcoef(dur, rel)[0, 1]), 3),
                  "corr_dur_radius": round(float(np.corrcoef(dur, rad)[0, 1]), 3),
                  "time_share_top1pct": round(float(np.sort(dur)[::-1][:len(dur) // 100].sum() / dur.sum()), 3)}))
