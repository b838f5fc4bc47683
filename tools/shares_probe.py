"""GPU box: what one rank of the sharded Jaccard costs on its own GPU (configs[3]).

For N in (1, 2, 4, 8) every part r of gs_jaccard_part_counts(r, N) is run
alone on the one GPU -- exactly the work rank r does on its own MI355X -- and
timed with HIP events (the library's profiler), as is the scatter
gs_jaccard_from_counts that every rank runs after the all-gather.  Prints one
JSON line: per N the slowest part, the scatter, the counts bytes each rank
sends, and the balance of the row cuts.

usage: shares_probe.py [SCALE] [REPS]"""
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

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
t = time.perf_counter()
ei = graphs.rmat(scale, 8, seed=0)
n = 1 << scale
gen = time.perf_counter() - t
ctx = Context(0)
dev = torch.device("cuda", 0)
ctx.set_graph_edge_index(n, torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev),
                         torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev))
del ei
eng = Engine(ctx)
whole = torch.empty(eng.nnz, dtype=torch.float64, device=dev)
eng.jaccard(out=whole)  # warm-up
out = {"workload": f"RMAT-{scale} sharded Jaccard, one rank's work per part", "E": eng.nnz,
       "graph_gen_s": round(gen, 2), "per_n": {}}


def timed(name, fn):
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    p = ctx.profile_read()
    ctx.profile(False)
    return p[name]["ms"] / p[name]["launches"]


out["whole_ms"] = round(timed("jaccard", lambda: eng.jaccard(out=whole)), 3)
for N in (1, 2, 4, 8):
    rc, oo = eng.jaccard_shares(N)
    sizes = np.diff(oo)
    stride = int(sizes.max())
    allc = torch.zeros(N * stride, dtype=torch.int32, device=dev)
    parts = []
    for r in range(N):
        buf = allc[r * stride: r * stride + max(int(sizes[r]), 1)]
        eng.jaccard_part_counts(r, N, out=buf)  # warm-up: the part's plan is kept per graph and rows
        parts.append(timed("jaccard", lambda: eng.jaccard_part_counts(r, N, out=buf)))
    res = torch.empty(eng.nnz, dtype=torch.float64, device=dev)
    scat = timed("jaccard_scatter", lambda: eng.jaccard_from_counts(N, allc, stride, out=res))
    same = bool(torch.equal(res.view(torch.int64), whole.view(torch.int64)))
    out["per_n"][N] = {"part_ms": [round(x, 3) for x in parts], "max_part_ms": round(max(parts), 3),
                       "scatter_ms": round(scat, 3), "counts_bytes_per_rank": int(4 * stride),
                       "allgather_bytes_total": int(4 * stride * N), "row_cut": rc.tolist(),
                       "bit_identical_to_whole": same}
print(json.dumps(out), flush=True)
