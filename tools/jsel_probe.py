"""GPU box: one rank's Jaccard-T work at N ranks (configs[3]) with the distributed select.

For N in (1, 2, 4, 8) the N parts of gs_jaccard_part_counts + gs_jsel_* run on N library
contexts of the one GPU, the all-reduces / all-gathers done here on the device; each
part's own calls are timed alone (HIP events of the library's profiler, and the wall
time of its synchronous calls, host overhead included) -- exactly the work rank r does
on its own MI355X.  Beside it, the replicated tail of the round-5 path that the select
replaces (the score scatter gs_jaccard_from_counts + the full gs_topk_mask on every
rank).  The exchange itself is modelled in DESIGN.md from its byte counts (printed).

usage: jsel_probe.py [SCALE] [KEEP] [REPS]"""
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
keep = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device("cuda", 0)
ei = graphs.rmat(scale, 8, seed=0)
n = 1 << scale
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
del ei


def engine():
    ctx = Context(0)
    ctx.set_graph_edge_index(n, src, dst)
    return ctx, Engine(ctx)


ctx0, e0 = engine()
nnz = e0.nnz
num_keep = int(nnz * keep)
whole = torch.empty(nnz, dtype=torch.float64, device=dev)
e0.jaccard(out=whole)
ref_mask = torch.empty(nnz, dtype=torch.uint8, device=dev)
_, cut0, nb0, nt0 = e0.topk_mask(whole, nnz, num_keep, False, out=ref_mask)
out = {"workload": f"RMAT-{scale} Jaccard-T (keep {keep}), one rank's work per part", "E": nnz,
       "num_keep": num_keep, "cut": cut0, "beyond": nb0, "tied": nt0, "per_n": {}}

prof_names = ("jaccard", "jsel_keys", "jsel_pass", "jsel_keep", "jsel_mask")
for N in (1, 2, 4, 8):
    ctxs, engs = zip(*[engine() for _ in range(N)])
    _, oo = engs[0].jaccard_shares(N)
    sizes = np.diff(oo)
    stride = int(sizes.max())
    counts = [torch.zeros(stride, dtype=torch.int32, device=dev) for _ in range(N)]
    hists = [torch.zeros(e.JSEL_BINS, dtype=torch.int64, device=dev) for e in engs]
    scores = [torch.empty(max(1, int(s)), dtype=torch.float64, device=dev) for s in sizes]
    s4 = (stride + 3) // 4
    kall = torch.zeros(N * s4, dtype=torch.uint8, device=dev)
    masks = [torch.empty(nnz, dtype=torch.uint8, device=dev) for _ in range(N)]
    wall = np.zeros(N)
    dev_ms = np.zeros(N)
    rec = {}
    for rep in range(reps + 1):  # the first round warms the plans and the slot table
        for c in ctxs:
            c.profile(True)
            c.profile_reset()
        w = np.zeros(N)

        def on(r, fn):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            v = fn()
            torch.cuda.synchronize(dev)
            w[r] += time.perf_counter() - t
            return v

        for r, e in enumerate(engs):
            on(r, lambda: e.jaccard_part_counts(r, N, out=counts[r]))
            on(r, lambda: e.jsel_begin(r, N, counts[r], num_keep, False, hists[r], scores[r]))
        left = engs[0].JSEL_PASSES
        while left:
            tot = torch.stack(hists).sum(0)
            for r, (h, e) in enumerate(zip(hists, engs)):
                h.copy_(tot)
                left = on(r, lambda: e.jsel_step(h))
        res = [on(r, lambda: e.jsel_result()) for r, e in enumerate(engs)]
        cut, nb, nt, _ = res[0]
        need = num_keep - nb
        tie_all = None
        if 0 < need < nt:
            pos = []
            for r, (e, x) in enumerate(zip(engs, res)):
                t_ = torch.zeros(max(1, x[3]), dtype=torch.int64, device=dev)
                on(r, lambda: e.jsel_tie_positions(t_))
                pos.append(t_[: x[3]])
            tie_all = torch.cat(pos)
        for r, e in enumerate(engs):
            on(r, lambda: e.jsel_keep(tie_all, nt, need, kall[r * s4:(r + 1) * s4]))
        for r, e in enumerate(engs):
            on(r, lambda: e.jsel_mask(N, kall, s4, masks[r]))
        if rep == 0:
            same = all(bool(torch.equal(m, ref_mask)) for m in masks)
            rec["mask_equals_one_gpu_topk"] = same
            rec["cut_beyond_tied"] = [cut, nb, nt]
            continue
        wall += w
        for r, c in enumerate(ctxs):
            p = c.profile_read()
            c.profile(False)
            dev_ms[r] += sum(p[k]["ms"] for k in prof_names if k in p)
            if r == 0:
                rec.setdefault("part0_kernels_ms", {})
                for k in prof_names:
                    if k in p:
                        rec["part0_kernels_ms"][k] = round(rec["part0_kernels_ms"].get(k, 0.0) + p[k]["ms"] / reps, 4)
    rec.update({"wall_ms_per_part": [round(x * 1e3 / reps, 3) for x in wall],
                "device_ms_per_part": [round(x / reps, 3) for x in dev_ms],
                "max_wall_ms": round(float(wall.max()) * 1e3 / reps, 3),
                "max_device_ms": round(float(dev_ms.max()) / reps, 3),
                "exchange_bytes": {"hist_allreduce_each": 8 * engs[0].JSEL_BINS, "passes": engs[0].JSEL_PASSES,
                                   "keep_allgather_total": int(N * s4),
                                   "ties_allgather_total": int(8 * nt) if tie_all is not None else 0}})
    out["per_n"][N] = rec
    del ctxs, engs, counts, masks
    torch.cuda.empty_cache()
    print(json.dumps({N: rec}), flush=True)
# the replicated tail of the round-5 path (per rank, every N): score scatter + full top-k
ctx0.profile(True)
ctx0.profile_reset()
for _ in range(reps):
    e0.topk_mask(whole, nnz, num_keep, False, out=ref_mask)
ctx0.synchronize()
p = ctx0.profile_read()
out["replicated_topk_ms"] = round(p["topk"]["ms"] / p["topk"]["launches"], 3)
print(json.dumps(out), flush=True)
