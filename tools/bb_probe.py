"""GPU box: what one rank of the sharded metric backbone costs on its own GPU
(configs[4], R-MAT-18 by default).

For N in (1, 2, 4, 8) every part r of gs_metric_backbone_part(r, N) is run alone
on the one GPU -- exactly the work rank r does on its own MI355X (the graph
build, witnesses and certificates are replicated; the searches of its source
rows are its own) -- and timed with HIP events (the library's profiler).  The
parts' keep bytes must add up to the whole mask.  Prints one JSON line: per N
every part's time, the slowest, and its ratio to the mean.

usage: bb_probe.py [SCALE] [REPS] [whole]   (whole: the one-part run only)"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gnn-sparsification-research_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from gsparse import graphs  # noqa: E402
from gsparse._lib import GS_DEVICE, Context  # noqa: E402
from gsparse.engine import Engine  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
whole_only = len(sys.argv) > 3 and sys.argv[3] == "whole"
t = time.perf_counter()
ei = graphs.rmat(scale, 8, seed=0)
n = 1 << scale
gen = time.perf_counter() - t
E = ei.shape[1]
dev = torch.device("cuda", 0)
ctx = Context(0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx.set_graph_edge_index(n, src, dst)
jac = Engine(ctx).jaccard()
# bench_backbone's costs: _scores_to_cost(Jaccard) in CSR order, [:E] (core.py:82-116)
sim = jac.copy()
p = sim / sim.max()
p[p <= 0] = p[p > 0].min() * 0.01
cost = (1.0 / p - 1.0)[:E]
w = torch.from_numpy(np.ascontiguousarray(cost)).to(dev)
relax = ctypes.c_int64(0)


def run(part, nparts, keep):
    ctx.call("gs_metric_backbone_part", n, E, src.data_ptr(), dst.data_ptr(), w.data_ptr(), w.numel(),
             GS_DEVICE, 1e-9, part, nparts, keep.data_ptr(), GS_DEVICE, ctypes.byref(relax))


PHASES = ("bb_build", "bb_witness", "bb_certify", "bb_search")
phase_ms = {}


def timed(fn):
    ctx.profile(True)
    ctx.profile_reset()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    p = ctx.profile_read()
    ctx.profile(False)
    phase_ms.clear()
    phase_ms.update({k: round(p[k]["ms"] / p[k]["launches"], 2) for k in PHASES if k in p})
    return p["metric_backbone"]["ms"] / p["metric_backbone"]["launches"]


whole = torch.empty(E, dtype=torch.uint8, device=dev)
run(0, 1, whole)  # warm-up
out = {"workload": f"RMAT-{scale} metric backbone, one rank's work per part", "E": E,
       "graph_gen_s": round(gen, 2), "whole_ms": round(timed(lambda: run(0, 1, whole)), 2),
       "kept": int(whole.sum().item()), "whole_phases_ms": dict(phase_ms), "per_n": {}}
print(json.dumps({"whole_ms": out["whole_ms"], "relaxations": relax.value,
                  "near_far": os.environ.get("GSPARSE_BB_NEARFAR", "default")}), flush=True)
for N in (() if whole_only else (2, 4, 8)):
    parts, rel, phases = [], [], []
    tot = torch.zeros(E, dtype=torch.int32, device=dev)
    for r in range(N):
        k = torch.empty(E, dtype=torch.uint8, device=dev)
        parts.append(timed(lambda: run(r, N, k)))
        rel.append(relax.value)
        phases.append(dict(phase_ms))
        tot += k.to(torch.int32)
    same = bool(torch.equal(tot.to(torch.uint8), whole)) and int(tot.max().item()) <= 1
    mean = sum(parts) / N
    out["per_n"][N] = {"part_ms": [round(x, 2) for x in parts], "max_part_ms": round(max(parts), 2),
                       "max_over_mean": round(max(parts) / mean, 4), "relaxations": rel,
                       "phases_ms_part0": phases[0],
                       "sum_equals_whole": same}
    print(json.dumps({N: out["per_n"][N]}), flush=True)
print(json.dumps(out), flush=True)
