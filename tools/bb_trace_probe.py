"""GPU box: per-batch timeline of the backbone's searches (GSPARSE_BB_TRACE), RMAT-18,
Jaccard costs.  One GPU (one range) and part 0..N-1 of the staged form at N (default
schedule), each part alone on the GPU as in tools/bb_stage_probe.py.  Per search launch:
its span, the workgroups' busy fraction, when fewer than half / a tenth of the
workgroups were still busy, and the longest batches.
usage: bb_trace_probe.py [SCALE] [N...]"""
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
from gsparse.distributed import backbone_phases  # noqa: E402
from gsparse.engine import Engine  # noqa: E402
from gsparse.metric_backbone import BackboneStages  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
Ns = [int(x) for x in sys.argv[2:]] or [1, 8]
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
w = torch.from_numpy(np.ascontiguousarray((1.0 / p - 1.0)[:E])).to(dev)
ei_d = torch.stack([src, dst])
stages = [BackboneStages(Context(0)) for _ in range(max(Ns))]


def run(N, fractions, path):
    st = stages[:N]
    K = [s.begin(ei_d, n, w, 1e-9, r, N) for r, s in enumerate(st)][0]
    if K and N > 1:
        Ds = [torch.empty(K * n, dtype=torch.float64, device=dev) for _ in range(N)]
        Cs = [torch.empty(K, dtype=torch.int32, device=dev) for _ in range(N)]
        for r in range(N):
            st[r].landmarks_io(Ds[r], Cs[r], out=True)
        D, C = torch.stack(Ds).min(0).values, torch.stack(Cs).max(0).values
        for r in range(N):
            st[r].landmarks_io(D, C, out=False)
    for r in range(N):
        st[r].certify(r, N)
    state = [torch.empty(E, dtype=torch.uint8, device=dev) for _ in range(N)]

    def exchange():
        if N == 1:
            return
        for r in range(N):
            st[r].state_io(state[r], out=True)
        m = torch.stack(state).max(0).values
        for r in range(N):
            st[r].state_io(m, out=False)

    exchange()
    nb = [s.plan() for s in st][0]
    os.environ["GSPARSE_BB_TRACE"] = path
    for b0, b1 in backbone_phases(nb, N, fractions):
        for r in range(N):
            st[r].search(b0, b1, r, N)
        exchange()
    os.environ.pop("GSPARSE_BB_TRACE")
    for r in range(N):
        st[r].finish()


def analyse(path, N):
    for line in open(path):
        d = json.loads(line)
        rec = np.array(d["rec"], dtype=np.float64)
        if rec.size == 0:
            continue
        t0, t1 = rec[:, 0], rec[:, 1]
        base = t0.min()
        t0, t1 = (t0 - base) / 100.0, (t1 - base) / 100.0  # constant clock 100 MHz -> us
        span = t1.max()
        dur = t1 - t0
        grid = d["grid"]
        # busy workgroups over time: sweep of start / end events
        ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
        ev = ev[np.argsort(ev[:, 0], kind="stable")]
        busy = np.cumsum(ev[:, 1])
        peak = busy.max()
        after = lambda frac: float(ev[np.flatnonzero(busy >= frac * peak)[-1], 0]) if np.any(busy >= frac * peak) else 0.0
        top = np.sort(dur)[::-1]
        print(json.dumps({"N": N, "part": d["part"], "range": [d["b0"], d["b1"]], "S": d["S"],
                          "grid": grid, "batches": int(rec.shape[0]), "span_ms": round(span / 1e3, 2),
                          "busy_frac": round(float(dur.sum() / (peak * span)), 3),
                          "last_half_busy_ms": round(after(0.5) / 1e3, 2),
                          "last_tenth_busy_ms": round(after(0.1) / 1e3, 2),
                          "longest_ms": [round(x / 1e3, 2) for x in top[:5]],
                          "mean_batch_ms": round(float(dur.mean()) / 1e3, 3),
                          "last_start_ms": round(float(t0.max()) / 1e3, 2)}), flush=True)


run(1, [], os.path.join(tempfile.gettempdir(), "bb_warm.jsonl"))  # warm-up
for N in Ns:
    path = os.path.join(os.environ.get("BB_TRACE_DIR", tempfile.gettempdir()), f"bb_trace_{N}.jsonl")
    if os.path.exists(path):
        os.remove(path)
    run(N, [] if N == 1 else None, path)
    analyse(path, N)
