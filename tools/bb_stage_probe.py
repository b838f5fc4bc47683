"""GPU box: one rank's work in the staged multi-rank metric backbone
(gsparse.distributed.sharded_backbone, gs_bb_*), R-MAT-18 by default (configs[4]).

For N in (1, 2, 4, 8) and each phase schedule, every part r of N runs its stages
on its own library context on the one GPU, one part at a time (exactly the work
rank r does on its own MI355X), and the exchanges between the stages are done
here on the device as the ranks' all-reduces would do them (landmark labels MIN,
completeness and column states MAX).  A stage's time at N is its slowest part's;
a rank's compute time is the sum over the stages.  Every schedule's mask must
equal the one-part mask.  Prints one JSON line per (schedule, N) and a summary.

usage: bb_stage_probe.py [SCALE] [SCHEDULES]   SCHEDULES: ';'-separated lists of
phase fractions, e.g. "0.5,0.8,0.95;0.9;" ('' = one search range)"""
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
from gsparse.distributed import backbone_phases  # noqa: E402
from gsparse.engine import Engine  # noqa: E402
from gsparse.metric_backbone import BackboneStages  # noqa: E402

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 18
sched_arg = sys.argv[2] if len(sys.argv) > 2 else "0.5,0.8,0.95;0.25,0.5,0.75,0.9,0.97;0.9;"
schedules = [[float(x) for x in s.split(",") if x.strip()] for s in sched_arg.split(";")]
t = time.perf_counter()
ei = graphs.rmat(scale, 8, seed=0) if scale > 0 else graphs.roman_like()
n = (1 << scale) if scale > 0 else 22_662
gen = time.perf_counter() - t
E = ei.shape[1]
dev = torch.device("cuda", 0)
ctx0 = Context(0)
src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
ctx0.set_graph_edge_index(n, src, dst)
jac = Engine(ctx0).jaccard()
# bench_backbone's costs: _scores_to_cost(Jaccard) in CSR order, [:E] (core.py:82-116)
sim = jac.copy()
p = sim / sim.max()
p[p <= 0] = p[p > 0].min() * 0.01
cost = (1.0 / p - 1.0)[:E]
w = torch.from_numpy(np.ascontiguousarray(cost)).to(dev)
ei_d = torch.stack([src, dst])
stages = [BackboneStages(Context(0)) for _ in range(8)]


def sync():
    torch.cuda.synchronize(dev)


def timed(fn):
    sync()
    t0 = time.perf_counter()
    r = fn()
    sync()
    return (time.perf_counter() - t0) * 1e3, r


def run(N, fractions):
    """One staged prune with N parts; returns (mask, per-stage slowest ms, per-stage all)."""
    st = stages[:N]
    ms = {}

    def stage(name, fn):
        times = []
        out = []
        for r in range(N):
            dt, o = timed(lambda: fn(r))
            times.append(dt)
            out.append(o)
        ms[name] = [round(x, 3) for x in times]
        return out

    K = stage("begin", lambda r: st[r].begin(ei_d, n, w, 1e-9, r, N))[0]
    if K and N > 1:
        Ds = [torch.empty(K * n, dtype=torch.float64, device=dev) for _ in range(N)]
        Cs = [torch.empty(K, dtype=torch.int32, device=dev) for _ in range(N)]
        for r in range(N):
            st[r].landmarks_io(Ds[r], Cs[r], out=True)
        D = torch.stack(Ds).min(0).values
        C = torch.stack(Cs).max(0).values
        for r in range(N):
            st[r].landmarks_io(D, C, out=False)
        del Ds, Cs
    stage("certify", lambda r: st[r].certify(r, N))
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
    nb = stage("plan", lambda r: st[r].plan())[0]
    for i, (b0, b1) in enumerate(backbone_phases(nb, N, fractions)):
        stage(f"search{i}[{b0},{b1})", lambda r: st[r].search(b0, b1, r, N))
        exchange()
    keeps = []
    for r in range(N):
        k = torch.empty(E, dtype=torch.uint8, device=dev)
        _, relax = st[r].finish(k)
        keeps.append((k, relax))
    sync()
    for k, _ in keeps[1:]:
        assert torch.equal(k, keeps[0][0])
    slow = {k: max(v) for k, v in ms.items()}
    return keeps[0][0], slow, ms, [r for _, r in keeps], nb


run(1, [])  # warm-up (allocations)
whole, slow1, _, rel1, nb1 = run(1, [])
base_ms = sum(slow1.values())
print(json.dumps({"workload": f"RMAT-{scale} metric backbone, staged, one part per rank", "E": E,
                  "graph_gen_s": round(gen, 2), "N": 1, "rank_ms": round(base_ms, 2),
                  "stages_ms": {k: round(v, 2) for k, v in slow1.items()}, "relaxations": rel1,
                  "nbatch": nb1, "kept": int(whole.sum().item())}), flush=True)
summary = {"N1_ms": round(base_ms, 2)}
for fr in schedules:
    for N in (2, 4, 8):
        mask, slow, allms, rel, nb = run(N, fr)
        assert torch.equal(mask, whole), (fr, N, int((mask != whole).sum().item()))
        tot = sum(slow.values())
        summary[f"{','.join(map(str, fr)) or 'one-range'}@N={N}"] = round(tot, 2)
        print(json.dumps({"phases": fr, "N": N, "rank_ms": round(tot, 2),
                          "speedup": round(base_ms / tot, 2),
                          "stages_ms": {k: round(v, 2) for k, v in slow.items()},
                          "parts_ms": allms, "relaxations": rel}), flush=True)
# search-geometry variants at N > 1 (argv[3]: ';'-separated "S:threads:slabs" triples;
# GSPARSE_BB_MULTI / _THREADS / _SLABS are read at plan time, per call)
variants = [v.split(":") for v in (sys.argv[3].split(";") if len(sys.argv) > 3 else []) if v]
for S, th, sl in variants:
    os.environ["GSPARSE_BB_MULTI"], os.environ["GSPARSE_BB_THREADS"] = S, th
    os.environ["GSPARSE_BB_SLABS"] = sl
    for N in (1, 4, 8):
        for fr in schedules[:1]:
            mask, slow, allms, rel, nb = run(N, fr)
            assert torch.equal(mask, whole), (S, th, sl, fr, N)
            tot = sum(slow.values())
            summary[f"S{S}/t{th}/slabs{sl} {','.join(map(str, fr))}@N={N}"] = round(tot, 2)
            print(json.dumps({"S": S, "threads": th, "slabs": sl, "phases": fr, "N": N,
                              "rank_ms": round(tot, 2),
                              "stages_ms": {k: round(v, 2) for k, v in slow.items()},
                              "relaxations": sum(rel), "nbatch": nb}), flush=True)
print(json.dumps({"summary": summary}), flush=True)
