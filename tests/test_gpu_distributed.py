"""Multi-GPU path on the device.

* The sharded scorers through a real RCCL ("nccl") process group with device
  tensors -- world 1 here (the test box has one GPU; bench.py's N-rank launch
  uses the same calls on 8) -- give the single-GPU bits.
* The Jaccard count shares (gs_jaccard_shares / gs_jaccard_part_counts /
  gs_jaccard_from_counts) equal the oracle's restatement of the layout and, put
  back together, the reference's Jaccard bit for bit, on graphs with rows in
  every owner-side class (LDS tables, bitmap rows, self-loops).
* Two ranks sharing the GPU over gloo run the whole N = 2 exchange with device
  compute on both ranks.
"""

import os
import socket

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal, load_golden

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


def _engine(gs, ei, n):
    data = gs.Data(edge_index=torch.from_numpy(np.ascontiguousarray(ei)), num_nodes=n)
    return gs.GraphSparsifier(data, "cuda:0")._engine


def _hub_graph():
    from test_gpu_parity import _hub_graph as hub

    return hub()


def _graphs():
    from gsparse import graphs

    ei, n = _hub_graph()
    yield "hub", ei, n
    yield "rmat14", graphs.rmat(14, 8, seed=5), 1 << 14
    g = load_golden("roman2000")
    yield "roman2000", g["edge_index"], int(g["num_nodes"])
    g = load_golden("karate_test")
    yield "karate_test", g["edge_index"], int(g["num_nodes"])


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_jaccard_count_shares_vs_oracle(gs, nparts):
    for name, ei, n in _graphs():
        ip, ix, _ = O.canonical_csr(ei, n)
        e = _engine(gs, ei, n)
        R, Oo = e.jaccard_shares(nparts)
        Rr, Or = O.jaccard_shares(ip, ix, nparts)
        assert np.array_equal(R, Rr) and np.array_equal(Oo, Or), name
        stride = max(1, int(np.diff(Oo).max()))
        allc = np.zeros(nparts * stride, dtype=np.uint32)
        dev = torch.zeros(nparts * stride, dtype=torch.int32, device="cuda:0")
        for p in range(nparts):
            c = e.jaccard_part_counts(p, nparts)
            assert np.array_equal(c, O.jaccard_part_counts(ip, ix, p, nparts)), (name, p)
            allc[p * stride: p * stride + len(c)] = c
            cnt = int(Oo[p + 1] - Oo[p])
            e.jaccard_part_counts(p, nparts, out=dev[p * stride: p * stride + max(cnt, 1)])
        ref = O.jaccard(ip, ix)
        assert bits_equal(e.jaccard_from_counts(nparts, allc, stride), ref), name
        out = torch.empty(e.nnz, dtype=torch.float64, device="cuda:0")
        e.jaccard_from_counts(nparts, dev, stride, out=out)
        assert bits_equal(out.cpu().numpy(), ref), name


@pytest.mark.parametrize("nparts", [127, 128, 200, 1000])
def test_jaccard_many_count_shares(gs, nparts):
    """More parts than one 128-thread block of cut threads (every cut
    must be written): the shares equal the oracle's and the parts' counts rebuild
    the reference's Jaccard."""
    for name, ei, n in _graphs():
        if name == "karate_test":
            continue
        ip, ix, _ = O.canonical_csr(ei, n)
        e = _engine(gs, ei, n)
        R, Oo = e.jaccard_shares(nparts)
        Rr, Or = O.jaccard_shares(ip, ix, nparts)
        assert np.array_equal(R, Rr) and np.array_equal(Oo, Or), name
        stride = max(1, int(np.diff(Oo).max()))
        allc = np.zeros(nparts * stride, dtype=np.uint32)
        for p in range(nparts):
            c = e.jaccard_part_counts(p, nparts)
            allc[p * stride: p * stride + len(c)] = c
        assert bits_equal(e.jaccard_from_counts(nparts, allc, stride), O.jaccard(ip, ix)), name
    with pytest.raises(ValueError):
        e.jaccard_part(0, 5000)


def test_jaccard_count_shares_errors(gs):
    g = load_golden("karate_test")
    e = _engine(gs, g["edge_index"], int(g["num_nodes"]))
    _, Oo = e.jaccard_shares(2)
    stride = int(np.diff(Oo).max())
    with pytest.raises(IndexError):
        e.jaccard_from_counts(2, np.zeros(2 * stride, dtype=np.uint32), stride - 1)
    with pytest.raises(ValueError):
        e.jaccard_part_counts(2, 2)
    d = load_golden("directed_dup")
    ed = _engine(gs, d["edge_index"], int(d["num_nodes"]))
    assert not ed.symmetric
    with pytest.raises(NotImplementedError):
        ed.jaccard_shares(2)


@pytest.fixture(scope="module")
def nccl_world1():
    """A real RCCL process group of one rank on cuda:0."""
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield dist
    finally:
        dist.destroy_process_group()


def test_nccl_sharded_scorers_equal_single_gpu(gs, nccl_world1):
    from gsparse import graphs
    from gsparse.distributed import (Comm, sharded_approx_er, sharded_backbone,
                                     sharded_edge_scores)

    assert nccl_world1.get_backend() == "nccl"
    comm = Comm(device=torch.device("cuda", 0))
    assert comm.device.type == "cuda" and comm.world == 1
    n = 12000
    ei = graphs.roman_like(n, 17500, seed=3)
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = gs.GraphSparsifier(data, "cuda:0")
    e = sp_._engine
    jac = sharded_edge_scores(e, comm, "jaccard")
    assert jac.is_cuda and bits_equal(jac.cpu().numpy(), e.jaccard())
    aa = sharded_edge_scores(e, comm, "adamic_adar")
    assert aa.is_cuda and bits_equal(aa.cpu().numpy(), e.adamic_adar())
    er = sharded_approx_er(e, comm, epsilon=0.9, max_cg_iters=60, blas_threads=8)
    assert er.is_cuda
    single = e.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=8)
    assert bits_equal(er.cpu().numpy(), single)
    cost = sp_._scores_to_cost(e.jaccard(), "jaccard")
    rows = O.csr_rows(e.indptr())
    ip, ix, _ = O.canonical_csr(ei, n)
    pos = np.searchsorted(rows * n + ix, ei[0] * n + ei[1])
    w = cost[pos]
    from gsparse.metric_backbone import backbone_mask

    keep = sharded_backbone(comm, ei, n, w)
    assert np.array_equal(keep, backbone_mask(ei, n, w, 1e-9))
    # the global top-k on the device after the all-gather (sharded_sparsify)
    from gsparse.distributed import sharded_sparsify

    E = ei.shape[1]
    jd = sharded_edge_scores(e, comm, "jaccard")
    for r in (0.9, 0.5, 0.1):
        m, info = sharded_sparsify(e, comm, jd, E, r, tie_break="stable")
        assert m.is_cuda and m.dtype == torch.bool
        ref = O.topk_mask(jd.cpu().numpy(), E, r, False, kind="stable")
        assert np.array_equal(m.cpu().numpy(), ref), r
        mn, _ = sharded_sparsify(e, comm, jd, E, r, tie_break="numpy")
        assert np.array_equal(mn.cpu().numpy(), O.topk_mask(jd.cpu().numpy(), E, r, False)), r


def _gloo_rank(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import gsparse
        from gsparse import graphs
        from gsparse.distributed import Comm, sharded_approx_er, sharded_edge_scores

        ei, n = _hub_graph()
        data = gsparse.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
        e = gsparse.GraphSparsifier(data, "cuda:0")._engine
        comm = Comm()
        jac_t = sharded_edge_scores(e, comm, "jaccard")
        jac = jac_t.numpy()
        from gsparse.distributed import sharded_sparsify

        E = ei.shape[1]
        masks = {r: sharded_sparsify(e, comm, jac_t, E, r, tie_break="stable")[0].numpy().copy()
                 for r in (0.8, 0.5, 0.2)}
        n2 = 12000
        ei2 = graphs.roman_like(n2, 17500, seed=3)
        e2 = gsparse.GraphSparsifier(gsparse.Data(edge_index=torch.from_numpy(ei2), num_nodes=n2),
                                     "cuda:0")._engine
        er = sharded_approx_er(e2, comm, epsilon=0.9, max_cg_iters=60, blas_threads=8).numpy()
        # the staged metric backbone (gs_bb_*): device compute on every rank, the
        # landmark labels and column states exchanged over gloo between the stages
        from gsparse.distributed import sharded_backbone

        bbs = {}
        for name, (eb, nb_) in _bb_graphs().items():
            w = _bb_costs(eb, nb_)
            bbs[name] = sharded_backbone(comm, eb, nb_, w)
            bbs[name + "-8phases"] = sharded_backbone(comm, eb, nb_, w, phases=[i / 8 for i in range(1, 8)],
                                                      method="staged")
            bbs[name + "-pairs"] = sharded_backbone(comm, eb, nb_, w, method="pairs")
        if rank == 0:
            q.put((jac, er, masks, bbs))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_sharing_the_gpu_over_gloo(gs, world, monkeypatch):
    """N ranks on the one GPU (device compute on every rank, gloo exchange):
    Jaccard count shares and ApproxER tree blocks (world 3: the non-power-of-two
    split) give the single-process bits."""
    import torch.multiprocessing as mp

    from gsparse import graphs

    monkeypatch.setenv("GSPARSE_REG_SPLIT", "0")  # ranks share the CUs
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    jac, er, masks, bbs = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    ei, n = _hub_graph()
    ip, ix, _ = O.canonical_csr(ei, n)
    ref = O.jaccard(ip, ix)
    assert bits_equal(jac, ref)
    # the global top-k after the exchange (core.py:229-240): N-rank kept set == one GPU
    # == np.argsort(kind='stable') of the reference's scores
    e1 = _engine(gs, ei, n)
    for r, m in masks.items():
        E = ei.shape[1]
        single, *_ = e1.topk_mask(ref, E, int(E * r), False)
        assert np.array_equal(m, single), r
        assert np.array_equal(m, O.topk_mask(ref, E, r, False, kind="stable")), r
    n2 = 12000
    ei2 = graphs.roman_like(n2, 17500, seed=3)
    e2 = _engine(gs, ei2, n2)
    assert bits_equal(er, e2.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=8))
    # the staged backbone over N ranks == one GPU's mask (metric_backbone.py:86-111)
    from gsparse.metric_backbone import backbone_mask

    for name, (eb, nb_) in _bb_graphs().items():
        ref = backbone_mask(eb, nb_, _bb_costs(eb, nb_))
        for key in (name, name + "-8phases", name + "-pairs"):
            assert np.array_equal(bbs[key], ref), (key, int((bbs[key] != ref).sum()))


def _bb_graphs():
    """The staged backbone's two search forms: the hub graph (n <= 65,536: one source
    per workgroup) and R-MAT-17 (8 sources per workgroup, reverse-column decisions)."""
    from gsparse import graphs

    ei, n = _hub_graph()
    return {"hub": (ei, n), "rmat17": (graphs.rmat(17, 8, seed=7), 1 << 17)}


def _bb_costs(ei, n):
    """_scores_to_cost(Jaccard) per edge_index column (sparsify_metric_backbone)."""
    ip, ix, _ = O.canonical_csr(ei, n)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    cost = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")
    return cost[np.searchsorted(rows * n + ix, ei[0].astype(np.int64) * n + ei[1])]


@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_staged_backbone_parts_vs_one_gpu(gs, nparts):
    """gs_bb_* with nparts parts, each on its own library context on the one GPU and
    the exchanges (labels MIN, flags / states MAX) done here on the device: the mask
    equals the single-call backbone's, under the default and a one-range schedule;
    also the relabeled R-MAT ids and the hub graph's one-source searches."""
    from gsparse._lib import Context
    from gsparse.distributed import backbone_phases
    from gsparse.metric_backbone import BackboneStages, backbone_mask

    dev = torch.device("cuda", 0)
    for name, (ei, n) in _bb_graphs().items():
        w = _bb_costs(ei, n)
        ref = backbone_mask(ei, n, w)
        E = ei.shape[1]
        for fractions in (None, []):
            st = [BackboneStages(Context(0)) for _ in range(nparts)]
            K = [s.begin(ei, n, w, 1e-9, r, nparts) for r, s in enumerate(st)][0]
            if K:
                Ds = [torch.empty(K * n, dtype=torch.float64, device=dev) for _ in st]
                Cs = [torch.empty(K, dtype=torch.int32, device=dev) for _ in st]
                for r, s in enumerate(st):
                    s.landmarks_io(Ds[r], Cs[r], out=True)
                D, C = torch.stack(Ds).min(0).values, torch.stack(Cs).max(0).values
                for s in st:
                    s.landmarks_io(D, C, out=False)
            for r, s in enumerate(st):
                s.certify(r, nparts)
            states = [torch.empty(E, dtype=torch.uint8, device=dev) for _ in st]

            def exchange():
                for r, s in enumerate(st):
                    s.state_io(states[r], out=True)
                m = torch.stack(states).max(0).values
                for s in st:
                    s.state_io(m, out=False)

            exchange()
            nbs = [s.plan() for s in st]
            assert len(set(nbs)) == 1
            for b0, b1 in backbone_phases(nbs[0], nparts, fractions):
                for r, s in enumerate(st):
                    s.search(b0, b1, r, nparts)
                exchange()
            for s in st:
                keep, _ = s.finish()
                assert np.array_equal(keep[:E].astype(bool), ref), (name, fractions)


@pytest.mark.parametrize("nparts", [1, 3])
def test_landmark_searches_spread_vs_one_workgroup(gs, nparts, monkeypatch):
    """The landmark searches of gs_bb_begin spread over the GPU (k_lm_round: W
    workgroups per landmark, one launch per round) reach the labels and completeness
    flags of one workgroup per landmark bit for bit (R-MAT-17, Jaccard costs), for
    every part's landmarks l = part (mod nparts)."""
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.metric_backbone import BackboneStages

    dev = torch.device("cuda", 0)
    ei, n = graphs.rmat(17, 8, seed=7), 1 << 17
    w = _bb_costs(ei, n)
    got = {}
    for coop in ("1", "0"):
        monkeypatch.setenv("GSPARSE_BB_LMCOOP", coop)
        for W in (("3", "64") if coop == "1" else ("0",)):
            monkeypatch.setenv("GSPARSE_BB_LMW", W)
            for r in range(nparts):
                st = BackboneStages(Context(0))
                K = st.begin(ei, n, w, 1e-9, r, nparts)
                assert K == 48
                D = torch.empty(K * n, dtype=torch.float64, device=dev)
                C = torch.empty(K, dtype=torch.int32, device=dev)
                st.landmarks_io(D, C, out=True)
                got[(coop, W, r)] = (D.cpu().numpy(), C.cpu().numpy())
    for r in range(nparts):
        D0, C0 = got[("0", "0", r)]
        mine = np.arange(r, 48, nparts)
        assert np.all(C0[mine] == 1)  # the one-workgroup searches ran dry
        assert np.isfinite(D0.reshape(n, 48)[:, mine]).any()
        for W in ("3", "64"):
            D1, C1 = got[("1", W, r)]
            assert np.array_equal(C1, C0), (W, r)
            assert bits_equal(D1, D0), (W, r)


def _jsel_parts(ei, n, nparts, r, low, dev):
    """gs_jsel_* with nparts parts, each on its own library context on the one GPU, the
    all-reduces / all-gathers done here on the device: (mask, info, own-pair scores)."""
    from gsparse._lib import Context
    from gsparse.engine import Engine

    engs = []
    for _ in range(nparts):
        ctx = Context(0)
        ctx.set_graph_edge_index(n, np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1]))
        engs.append(Engine(ctx))
    nnz = engs[0].nnz
    _, Oo = engs[0].jaccard_shares(nparts)
    sizes = np.diff(Oo)
    stride = max(1, int(sizes.max()))
    num_keep = int(nnz * r)
    hists, scores = [], []
    for p, e in enumerate(engs):
        c = torch.zeros(stride, dtype=torch.int32, device=dev)
        e.jaccard_part_counts(p, nparts, out=c)
        h = torch.zeros(e.JSEL_BINS, dtype=torch.int64, device=dev)
        s = torch.empty(max(1, int(sizes[p])), dtype=torch.float64, device=dev)
        e.jsel_begin(p, nparts, c, num_keep, low, h, s)
        hists.append(h)
        scores.append(s[: int(sizes[p])])
    left = engs[0].JSEL_PASSES
    while left:
        tot = torch.stack(hists).sum(0)
        lefts = set()
        for h, e in zip(hists, engs):
            h.copy_(tot)
            lefts.add(e.jsel_step(h))
        assert len(lefts) == 1
        left = lefts.pop()
    res = [e.jsel_result() for e in engs]
    assert len({x[:3] for x in res}) == 1  # every part agrees on the cut
    cut, nb, nt, _ = res[0]
    need = num_keep - nb
    tie_all = None
    if 0 < need < nt:
        pos = []
        for e, x in zip(engs, res):
            t = torch.zeros(max(1, x[3]), dtype=torch.int64, device=dev)
            e.jsel_tie_positions(t)
            pos.append(t[: x[3]])
        tie_all = torch.cat(pos)
        assert tie_all.numel() == nt
    s4 = (stride + 3) // 4
    kall = torch.zeros(nparts * s4, dtype=torch.uint8, device=dev)
    for p, e in enumerate(engs):
        e.jsel_keep(tie_all, nt, need, kall[p * s4:(p + 1) * s4])
    masks = []
    for e in engs:
        m = torch.empty(nnz, dtype=torch.uint8, device=dev)
        e.jsel_mask(nparts, kall, s4, m)
        masks.append(m.cpu().numpy().astype(bool))
    for m in masks[1:]:
        assert np.array_equal(m, masks[0])
    info = {"cut": cut, "beyond": nb, "tied": nt, "need": need}
    return masks[0], info, [s.cpu().numpy() for s in scores]


def _tie_graph():
    """Many equal scores: a union of disjoint cliques and stars (Jaccard 1 inside a
    clique, 0 / small values on the stars), plus a self-loop."""
    rng = np.random.default_rng(11)
    edges = []
    base = 0
    for _ in range(40):
        k = int(rng.integers(3, 7))
        nodes = np.arange(base, base + k)
        for a in nodes:
            for b in nodes:
                if a != b:
                    edges.append((a, b))
        base += k
    for _ in range(30):
        k = int(rng.integers(2, 9))
        for leaf in range(1, k + 1):
            edges += [(base, base + leaf), (base + leaf, base)]
        base += k + 1
    edges.append((0, 0))
    ei = np.asarray(edges, dtype=np.int64).T
    return np.ascontiguousarray(ei), base


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_distributed_jaccard_select_vs_one_gpu(gs, nparts):
    """gs_jsel_* (Jaccard-T without the score exchange, core.py:229-240): for every
    retention ratio and both directions the parts' mask equals one GPU's gs_topk_mask on
    the whole scores (= np.argsort(kind='stable')), the cut / beyond / tied counts match,
    and every part's own-pair scores are the reference's Jaccard at its owner entries."""
    from gsparse import graphs

    dev = torch.device("cuda", 0)
    cases = [("tie", *_tie_graph()), ("hub", *_hub_graph()), ("rmat14", graphs.rmat(14, 8, seed=5), 1 << 14)]
    g = load_golden("roman2000")
    cases.append(("roman2000", g["edge_index"], int(g["num_nodes"])))
    for name, ei, n in cases:
        ip, ix, _ = O.canonical_csr(ei, n)
        ref = O.jaccard(ip, ix)
        nnz = len(ref)
        e1 = _engine(gs, ei, n)
        rows = O.csr_rows(ip)
        deg = np.diff(ip)
        own = np.nonzero((deg[rows] > deg[ix]) | ((deg[rows] == deg[ix]) & (rows <= ix)))[0]
        _, Oo = e1.jaccard_shares(nparts)
        for r in (0.9, 0.5, 0.2, 0.05):
            for low in (False, True):
                m, info, sc = _jsel_parts(ei, n, nparts, r, low, dev)
                single, cut, nb, nt = e1.topk_mask(ref, nnz, int(nnz * r), low)
                assert np.array_equal(m, single), (name, r, low, info)
                assert np.array_equal(m, O.topk_mask(ref, nnz, r, low, kind="stable")), (name, r, low)
                assert (info["beyond"], info["tied"]) == (nb, nt) and info["cut"] == cut, (name, r, low)
        for p in range(nparts):  # the own-pair scores (last case's parts) = the reference's
            assert bits_equal(sc[p], ref[own[Oo[p]:Oo[p + 1]]]), (name, p)


def test_nccl_jaccard_topk_world1(gs, nccl_world1):
    """sharded_jaccard_topk through a real RCCL group (world 1, device tensors): the
    mask equals one GPU's stable top-k; tie_break="numpy" equals the reference's
    np.argsort rule on an ambiguous cut."""
    from gsparse import graphs
    from gsparse.distributed import Comm, sharded_jaccard_topk

    comm = Comm(device=torch.device("cuda", 0))
    ei, n = graphs.rmat(14, 8, seed=5), 1 << 14
    e = _engine(gs, ei, n)
    ip, ix, _ = O.canonical_csr(ei, n)
    ref = O.jaccard(ip, ix)
    nnz = len(ref)
    for r in (0.8, 0.5, 0.2):
        m, info, sc = sharded_jaccard_topk(e, comm, r, tie_break="stable")
        assert m.is_cuda
        assert np.array_equal(m[:nnz].cpu().numpy().astype(bool), O.topk_mask(ref, nnz, r, False, kind="stable")), r
        mn, info_n, _ = sharded_jaccard_topk(e, comm, r, tie_break="numpy")
        assert np.array_equal(mn[:nnz].cpu().numpy().astype(bool), O.topk_mask(ref, nnz, r, False)), r
    m, info, _ = sharded_jaccard_topk(e, comm, 1.0)
    assert bool(m[:nnz].all()) and info["beyond"] == nnz
