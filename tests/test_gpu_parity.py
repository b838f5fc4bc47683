"""GPU parity: libgsparse.so (through the drop-in API and the C ABI) vs the
reference's golden vectors and the pinned oracle.

Bar: bit-identical float64 scores for Jaccard / Adamic-Adar / degree /
FeatCos / ApproxER (the device reproduces NumPy's, SciPy's and OpenBLAS's
operation order -- golden ApproxER vectors were made with
OPENBLAS_NUM_THREADS=1, so the device runs with blas_threads=1 here);
identical keep masks for top-k (numpy tie mode), the metric backbone, the
sampled and degree-aware selections.
"""

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import (EXACT_ER_ATOL, bits_equal, exact_er_golden, exact_er_names, golden_features,
                      golden_names, load_golden)

pytestmark = pytest.mark.gpu

SMALL = golden_names(include_big=False)


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


def make(gs, g, tie_break="numpy", with_x=True):
    x = golden_features(g) if with_x else None
    data = gs.Data(edge_index=torch.from_numpy(g["edge_index"]),
                   x=torch.from_numpy(x) if x is not None else None,
                   num_nodes=int(g["num_nodes"]))
    return gs.GraphSparsifier(data, "cpu", tie_break=tie_break), data


@pytest.mark.parametrize("name", SMALL)
def test_scores_bit_exact(gs, name):
    g = load_golden(name)
    sp_, _ = make(gs, g)
    a = sp_.adj
    assert np.array_equal(a.indptr, g["indptr"]) and np.array_equal(a.indices, g["indices"])
    assert bits_equal(a.data, g["data"])
    for m in ["jaccard", "adamic_adar", "degree"]:
        assert bits_equal(sp_.compute_scores(m), g[f"scores_{m}"]), m
    if "scores_feature_cosine" in g:
        assert bits_equal(sp_.compute_scores("feature_cosine"), g["scores_feature_cosine"])


@pytest.mark.parametrize("name", SMALL)
def test_approx_er_bit_exact(gs, name):
    g = load_golden(name)
    sp_, _ = make(gs, g, with_x=False)
    er = sp_._engine.approx_er(blas_threads=1)
    ref = g["scores_approx_er"]
    assert bits_equal(er, ref), float(np.max(np.abs(er - ref) / np.abs(ref)))


@pytest.mark.parametrize("mode", ["0", "1", "2", "3", "4", "5", "5n", "5r"])
@pytest.mark.parametrize("name", ["karate_csr", "rmat10", "directed_dup", "roman2000"])
def test_approx_er_all_cg_modes(gs, name, mode, monkeypatch):
    """q recomputed in the update kernel (0), stored by the fused p/q kernel (1),
    split p stream + SpMV (2, 3), the resident per-column solver (4), or the
    register-resident one (5: one BLAS chunk here, 8 threads per chain; 5n: its
    256-thread form; 5r: q recomputed instead of kept in registers) -- the same bits in every mode."""
    if mode == "5n":
        mode = "5"
        monkeypatch.setenv("GSPARSE_REG_NT", "256")
    if mode == "5r":  # 512-thread form with q recomputed in the r update, x in registers
        mode = "5"
        monkeypatch.setenv("GSPARSE_REG_QR", "0")
    monkeypatch.setenv("GSPARSE_CG_MODE", mode)
    g = load_golden(name)
    sp_, _ = make(gs, g, with_x=False)
    assert bits_equal(sp_._engine.approx_er(blas_threads=1), g["scores_approx_er"])


@pytest.fixture(scope="module")
def chunked_er():
    """n > 10000, so OpenBLAS splits every ddot into T thread chunks; a short
    maxiter keeps the oracle's CG (oracle.c) to seconds."""
    from gsparse import graphs

    n = 12000
    ei = graphs.roman_like(n, 17500, seed=3)
    # the same graph with every 7th edge doubled: multiplicity-2 entries, so the
    # resident solver's unit-weight SELL form does not apply
    dup = np.concatenate([ei, ei[:, ::7]], axis=1)
    # unit weights with a few rows wider than the SpMV's first 8 entries (its tail loop)
    rng = np.random.default_rng(11)
    extra = [(h, int(v)) for h, k in ((5, 40), (6001, 13), (11990, 9)) for v in rng.choice(n, k, replace=False)
             if v != h]
    ex = np.array(extra, dtype=np.int64).T
    hub = O.coalesce(np.concatenate([ei, ex], axis=1), n)
    out = {}
    for gname, e in (("unit", ei), ("dup", dup), ("hub", hub)):
        ip, ix, d = O.canonical_csr(e, n)
        out[gname] = (e, {t: O.approx_er(ip, ix, d, n, epsilon=0.9, max_cg_iters=60, impl="c",
                                         blas_threads=t) for t in (3, 8)})
    return n, out


@pytest.mark.parametrize("env", [{"GSPARSE_CG_MODE": "0"}, {"GSPARSE_CG_MODE": "1"},
                                 {"GSPARSE_CG_MODE": "3"}, {"GSPARSE_CG_MODE": "4"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_ELL": "1"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_QLDS": "0"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_CG_SLOTS": "7"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_UNIT": "0",
                                  "GSPARSE_RES_ELL": "1"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_STAB": "0"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_RBW": "44"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_RBW": "44",
                                  "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_DCOUNT": "0"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_RBW": "26"},
                                 {"GSPARSE_CG_MODE": "4", "GSPARSE_RES_RBW": "28"},
                                 {"GSPARSE_CG_MODE": "5"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_RES_DCOUNT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_CG_SLOTS": "7"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_KEEP": "40"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_KEEP": "0",
                                  "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_NT": "256"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_NT": "256",
                                  "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_NT": "256",
                                  "GSPARSE_REG_KEEP": "40"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_QR": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_QR": "0", "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_QR": "0", "GSPARSE_REG_KEEP": "40"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_SPLIT": "2"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_SPLIT": "3"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_SPLIT": "4", "GSPARSE_RES_UNIT": "0"},
                                 {"GSPARSE_CG_MODE": "5", "GSPARSE_REG_SPLIT": "2", "GSPARSE_REG_SPLIT_SPIN": "0"}],
                         ids=["m0", "m1", "m3", "m4", "m4-ell", "m4-q-global", "m4-7slots",
                              "m4-weighted-sell", "m4-weighted-ell", "m4-slices-global",
                              "m4-rb4w4", "m4-rb4w4-weighted", "m4-diag-loaded", "m4-w6", "m4-w8",
                              "m5", "m5-weighted", "m5-diag-loaded", "m5-7slots", "m5-p-global",
                              "m5-p-all-global-weighted", "m5-narrow", "m5-narrow-weighted",
                              "m5-narrow-p-global", "m5-q-recomputed", "m5-q-recomputed-weighted",
                              "m5-q-recomputed-p-global", "m5-split2", "m5-split3", "m5-split4-weighted",
                              "m5-split2-gives-up"])
@pytest.mark.parametrize("threads", [3, 8])
@pytest.mark.parametrize("graph", ["unit", "dup", "hub"])
def test_approx_er_blas_chunks_vs_oracle(gs, chunked_er, graph, threads, env, monkeypatch):
    """T-chunk ddot order (T = 3, 8) in every CG mode, bit-identical to the oracle."""
    for k_, v in env.items():
        monkeypatch.setenv(k_, v)
    n, graphs_ = chunked_er
    ei, ref = graphs_[graph]
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = gs.GraphSparsifier(data, "cpu")
    er = sp_._engine.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=threads)
    assert bits_equal(er, ref[threads])


@pytest.mark.parametrize("mode", ["0", "1", "3", "4", "5", "5s"])
def test_er_column_blocks_in_every_mode(gs, chunked_er, mode, monkeypatch):
    """A rank's column block [col0, col1) (the N-GPU split) solved alone, in the
    batched and the resident solver: the blocks' partial sums, added along the
    pairwise tree, equal the whole -- and the whole equals the oracle (5s: every
    column solved by 2 workgroups, k_cg_regwide's split form)."""
    if mode == "5s":
        mode = "5"
        monkeypatch.setenv("GSPARSE_REG_SPLIT", "2")
    monkeypatch.setenv("GSPARSE_CG_MODE", mode)
    n, graphs_ = chunked_er
    ei, ref = graphs_["unit"]
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    e = sp_._engine
    k = gs.engine.jl_dim(n, 0.9)
    e.er_prepare(k)
    e.er_project_device(np.random.default_rng(42), k)
    b = gs.engine.er_split(k, 2)
    sums = []
    for i in range(2):  # each block solved on its own, as one rank would
        e.er_solve(int(b[i]), int(b[i + 1]), 60, 1e-6, 8)
        sums.append(e.er_scores(int(b[i]), int(b[i + 1]), finalize=False))
    tot = 0.0 + (sums[0] + sums[1])
    tot = np.maximum(np.nan_to_num(tot, nan=1e-10, posinf=1e-10, neginf=1e-10), 1e-10)
    assert bits_equal(tot, ref[8])


def test_split_tail_in_offset_column_blocks(gs, chunked_er, monkeypatch):
    """Column blocks that start past column 0 and leave a split last round (each
    block ~325 columns: one whole round of 256, then ~69 columns in parts; the automatic
    split, GSPARSE_REG_SPLIT_AUTO=1) give the same bits as the whole solve with the split
    form disabled."""
    monkeypatch.setenv("GSPARSE_CG_MODE", "5")
    n, graphs_ = chunked_er
    ei, _ = graphs_["unit"]
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    e = sp_._engine
    k = gs.engine.jl_dim(n, 0.59)
    e.er_prepare(k)
    e.er_project_device(np.random.default_rng(42), k)
    monkeypatch.setenv("GSPARSE_REG_SPLIT", "0")
    e.er_solve(0, k, 40, 1e-6, 8)
    whole = e.er_scores(0, k, finalize=False).copy()
    monkeypatch.delenv("GSPARSE_REG_SPLIT")
    monkeypatch.setenv("GSPARSE_REG_SPLIT_AUTO", "1")  # the automatic split (off by default)
    b = gs.engine.er_split(k, 2)
    assert 256 < int(b[1]) - int(b[0]) <= 384 and 256 < int(b[2]) - int(b[1]) <= 384
    sums = []
    for i in range(2):
        e.er_solve(int(b[i]), int(b[i + 1]), 40, 1e-6, 8)
        sums.append(e.er_scores(int(b[i]), int(b[i + 1]), finalize=False).copy())
    e.er_solve(0, k, 40, 1e-6, 8)  # whole range, split tail on
    assert bits_equal(e.er_scores(0, k, finalize=False), whole)
    # the blocks' partial sums are pairwise-tree halves of the whole sum
    assert bits_equal(0.0 + (sums[0] + sums[1]), whole)


def test_approx_er_roman_full_bit_exact(gs):
    """configs[1] size (n=22,662, E=65,854, k=2,674, 500 CG iterations per column)."""
    g = load_golden("roman_full")
    sp_, _ = make(gs, g, with_x=False)
    er = sp_._engine.approx_er(blas_threads=1)
    ref = g["scores_approx_er"]
    rel = float(np.max(np.abs(er - ref) / np.abs(ref)))
    assert rel <= 1e-5, rel  # north_star tolerance
    assert bits_equal(er, ref), rel
    it = sp_._engine.er_iterations()
    assert it.shape == (2674,)


def test_roman_full_structural_and_featcos(gs):
    g = load_golden("roman_full")
    sp_, _ = make(gs, g)
    for m in ["jaccard", "adamic_adar", "degree", "feature_cosine"]:
        assert bits_equal(sp_.compute_scores(m), g[f"scores_{m}"]), m


def test_weighted_karate_module_functions(gs):
    import scipy.sparse as sp

    z = load_golden("karate_weighted")
    n = int(z["num_nodes"])
    adj = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))
    assert bits_equal(gs.calculate_jaccard_scores(adj), z["scores_jaccard"])
    assert bits_equal(gs.calculate_adamic_adar_scores(adj), z["scores_adamic_adar"])
    er = gs.calculate_approx_effective_resistance_scores(adj, epsilon=0.3, seed=42)
    assert bits_equal(er, z["scores_approx_er"])
    from scipy.stats import spearmanr

    assert spearmanr(z["scores_effective_resistance"], er)[0] > 0.5


@pytest.mark.parametrize("name", SMALL)
def test_topk_masks(gs, name):
    g = load_golden(name)
    sp_n, _ = make(gs, g, "numpy")
    sp_s, _ = make(gs, g, "stable")
    metrics = ["jaccard", "adamic_adar", "degree", "approx_er"] + \
        (["feature_cosine"] if "scores_feature_cosine" in g else [])
    E = g["edge_index"].shape[1]
    for m in metrics:
        sp_n._score_cache[sp_n._normalize_metric_name(m)] = g[f"scores_{m}"]
        sp_s._score_cache[sp_s._normalize_metric_name(m)] = g[f"scores_{m}"]
        for r in [0.9, 0.8, 0.6, 0.5, 0.4, 0.2]:
            for low in (0, 1):
                _, mask = sp_n.sparsify(m, r, return_mask=True, keep_lowest=bool(low))
                assert np.array_equal(mask.numpy(), g[f"mask_{m}_{r}_{low}"]), (m, r, low)
                sd, mask_s = sp_s.sparsify(m, r, return_mask=True, keep_lowest=bool(low))
                ref_s = O.topk_mask(g[f"scores_{m}"], E, r, bool(low), kind="stable")
                assert np.array_equal(mask_s.numpy(), ref_s), (m, r, low)
                assert sd.edge_index.shape[1] == int(mask_s.sum())


@pytest.mark.parametrize("name", SMALL)
def test_backbone(gs, name):
    g = load_golden(name)
    sp_, data = make(gs, g, with_x=False)
    for m in ["jaccard", "adamic_adar", "degree", "approx_er"]:
        cost = g[f"cost_{m}"]
        if f"backbone_{m}_error" in g:
            with pytest.raises(IndexError):
                gs.compute_metric_backbone(data, cost, epsilon=1e-9, verbose=False)
            continue
        _, st = gs.compute_metric_backbone(data, cost, epsilon=1e-9, verbose=False)
        assert np.array_equal(st["keep_mask"], g[f"backbone_{m}"]), m
        assert st["edges_metric"] == int(g[f"backbone_{m}_metric"])


@pytest.mark.parametrize("name", ["karate_test", "roman2000", "cora_like"])
def test_sampled_degree_aware(gs, name):
    g = load_golden(name)
    sp_, _ = make(gs, g, with_x=False)
    for m in ["jaccard", "degree"]:
        sp_._score_cache[m] = g[f"scores_{m}"]
        for r in (0.5, 0.2):
            _, mk = sp_.sparsify_sampled(m, r, seed=42, return_mask=True)
            assert np.array_equal(mk.numpy(), g[f"sampled_{m}_{r}"])
            _, mk = sp_.sparsify_degree_aware(m, r, return_mask=True)
            assert np.array_equal(mk.numpy(), g[f"degaware_{m}_{r}"])


# ----------------------------------------------------------------- larger sizes
@pytest.fixture(scope="module")
def rmat14():
    from gsparse import graphs

    ei = graphs.rmat(14, 8, seed=5)
    n = 1 << 14
    ip, ix, d = O.canonical_csr(ei, n)
    return ei, n, ip, ix, d


def test_rmat14_vs_oracle(gs, rmat14):
    ei, n, ip, ix, d = rmat14
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = gs.GraphSparsifier(data, "cpu")
    assert np.array_equal(sp_.adj.indptr, ip) and np.array_equal(sp_.adj.indices, ix)
    assert bits_equal(sp_.compute_scores("jaccard"), O.jaccard(ip, ix))
    assert bits_equal(sp_.compute_scores("adamic_adar"), O.adamic_adar(ip, ix))
    # edge-range partition (the multi-GPU split) concatenates to the whole
    e = sp_._engine
    cuts = [0, 1000, 77777, e.nnz]
    parts = [e.jaccard(cuts[i], cuts[i + 1]) for i in range(3)]
    assert bits_equal(np.concatenate(parts), sp_.compute_scores("jaccard"))


def _column_costs(ei, n):
    """Jaccard costs (_scores_to_cost) per edge_index column: the CSR entry of
    each column's (u, v), so graphs with duplicate columns get E weights."""
    ip, ix, _ = O.canonical_csr(ei, n)
    rows = np.repeat(np.arange(n), np.diff(ip))
    cost_csr = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")
    pos = np.searchsorted(rows.astype(np.int64) * n + ix, ei[0].astype(np.int64) * n + ei[1])
    return cost_csr[pos]


def _hub_graph():
    """RMAT-14 plus hubs in every Jaccard row class of gs_jaccard.hip (LDS tables
    of 2K / 8K / 32K slots and the > 16384 bitmap rows), hub-hub edges and
    self-loops; symmetrised."""
    from gsparse import graphs

    n = 60000
    parts = [graphs.rmat(14, 8, seed=11)]
    for hub, lo, cnt in [(1, 100, 20000), (2, 50, 10000), (3, 7, 3000), (4, 1000, 800),
                         (5, 30000, 17000)]:
        leaves = np.arange(lo, lo + cnt, dtype=np.int64)
        parts.append(np.stack([np.full(cnt, hub), leaves]))
    parts.append(np.array([[1, 2, 3, 1, 5], [2, 3, 4, 5, 2]], dtype=np.int64))
    loops = np.arange(0, 12, dtype=np.int64)
    parts.append(np.stack([loops, loops]))
    ei = np.concatenate(parts, axis=1)
    ei = np.concatenate([ei, ei[::-1]], axis=1)
    return ei, n


def test_jaccard_owner_hash_classes_vs_oracle(gs, monkeypatch):
    ei, n = _hub_graph()
    ip, ix, _ = O.canonical_csr(ei, n)
    assert np.diff(ip).max() > 16384
    ref = O.jaccard(ip, ix)
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = gs.GraphSparsifier(data, "cpu")
    e = sp_._engine
    assert e.symmetric
    assert bits_equal(e.jaccard(), ref)
    monkeypatch.setenv("GSPARSE_JACCARD", "merge")
    assert bits_equal(e.jaccard(), ref)


@pytest.mark.parametrize("qdmax", [None, "0", "1"])
@pytest.mark.parametrize("graph", ["hub60k", "spread3m"])
def test_jaccard_quotient_tables_vs_oracle(gs, monkeypatch, graph, qdmax):
    """The 16-bit quotient tables of row classes 1-3 (gs_jaccard.hip k_jac_hashq):
    hubs in every class, ids of 16 bits (hub60k) and of 22 bits (spread3m: the
    remainder width of RMAT-22), and -- GSPARSE_JAC_QDMAX -- the largest encodable
    bucket distance cut to 0 / 1, so tasks overflow and probe the sorted list."""
    rng = np.random.default_rng(5)
    if graph == "hub60k":
        ei, n = _hub_graph()
        extra = np.stack([np.full(6000, 6), np.arange(40000, 46000)])
    else:
        n = 3_000_000
        ei = np.zeros((2, 0), dtype=np.int64)
        extra = np.zeros((2, 0), dtype=np.int64)
    hubs = []
    for hub, cnt in [(11, 2500), (12, 4000), (13, 7000), (14, 12000), (15, 15000)]:
        lv = rng.choice(min(n, 200000) if graph == "hub60k" else n, cnt, replace=False)
        hubs.append(np.stack([np.full(cnt, hub), lv]))
    # shared leaves between hubs, so intersections are non-trivial
    shared = rng.choice(n, 3000, replace=False)
    for hub in (12, 13, 14):
        hubs.append(np.stack([np.full(3000, hub), shared]))
    e2 = np.concatenate([ei, extra] + [h % n for h in hubs], axis=1)
    e2 = np.concatenate([e2, e2[::-1]], axis=1)
    ip, ix, _ = O.canonical_csr(e2, n)
    deg = np.diff(ip)
    for lo, hi in [(1024, 4096), (4096, 8192), (8192, 16384)]:
        assert ((deg > lo) & (deg <= hi)).any(), (lo, hi)
    ref = O.jaccard(ip, ix)
    if qdmax is not None:
        monkeypatch.setenv("GSPARSE_JAC_QDMAX", qdmax)
    data = gs.Data(edge_index=torch.from_numpy(e2), num_nodes=n)
    e = gs.GraphSparsifier(data, "cpu")._engine
    assert bits_equal(e.jaccard(), ref)


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
def test_jaccard_parts_sum_to_whole(gs, nparts):
    ei, n = _hub_graph()
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    e = gs.GraphSparsifier(data, "cpu")._engine
    whole = e.jaccard()
    parts = [e.jaccard_part(p, nparts) for p in range(nparts)]
    tot = np.zeros_like(whole)
    for p in parts:
        tot = tot + p
    assert bits_equal(tot, whole)
    # every entry has exactly one contributing part
    assert np.array_equal(sum((p != 0).astype(int) for p in parts), (whole != 0).astype(int))
    # directed graph: edge ranges
    g = load_golden("directed_dup")
    d = gs.Data(edge_index=torch.from_numpy(g["edge_index"]), num_nodes=int(g["num_nodes"]))
    ed = gs.GraphSparsifier(d, "cpu")._engine
    tot = sum(ed.jaccard_part(p, nparts) for p in range(nparts))
    assert bits_equal(tot, g["scores_jaccard"])


@pytest.mark.parametrize("relabel", ["0", "1"])
@pytest.mark.parametrize("name", ["karate_test", "directed_dup", "rmat10", "roman2000"])
def test_backbone_relabel_either_way(gs, name, relabel, monkeypatch):
    """The degree-ordered node relabeling (automatic for graphs without id locality)
    forced on and off: the same keep masks as the reference."""
    monkeypatch.setenv("GSPARSE_BB_RELABEL", relabel)
    g = load_golden(name)
    _, data = make(gs, g, with_x=False)
    for m in ["jaccard", "approx_er"]:
        if f"backbone_{m}_error" in g:
            continue
        _, st = gs.compute_metric_backbone(data, g[f"cost_{m}"], epsilon=1e-9, verbose=False)
        assert np.array_equal(st["keep_mask"], g[f"backbone_{m}"]), (m, relabel)


def test_backbone_rmat12_vs_oracle(gs):
    from gsparse import graphs

    ei = graphs.rmat(12, 8, seed=2)
    n = 1 << 12
    ip, ix, d = O.canonical_csr(ei, n)
    cost = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")
    keep_ref = O.metric_backbone(ei, n, cost)
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    _, st = gs.compute_metric_backbone(data, cost, verbose=False)
    assert np.array_equal(st["keep_mask"], keep_ref)


@pytest.mark.parametrize("graph", ["rmat14", "hub", "roman"])
@pytest.mark.parametrize("off", [("GSPARSE_BB_LANDMARKS",), ("GSPARSE_BB_LOCALLB",), ("+GSPARSE_BB_MITM",),
                                 ("+GSPARSE_BB_MITM", "GSPARSE_BB_MITM_LM"),
                                 ("GSPARSE_BB_LANDMARKS", "GSPARSE_BB_LOCALLB")])
def test_backbone_certificates_match_plain_search(gs, graph, off, monkeypatch):
    """Landmark / degree-1 / local-bound certificates (default) vs the search with the
    landmark certificates, the local bounds (least other edge weights; the 3- and 4-edge
    bounds of the witness pass) or both off, and with the pair (meet-in-the-middle)
    certificate on, its landmarks blocked or not (GSPARSE_BB_LANDMARKS=0,
    GSPARSE_BB_LOCALLB=0, GSPARSE_BB_MITM=1, GSPARSE_BB_MITM_LM=0; the plain 2-hop
    witness + bounded search is pinned to the oracle above)."""
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    if graph == "rmat14":
        ei, n = graphs.rmat(14, 8, seed=3), 1 << 14
    elif graph == "hub":
        ei, n = _hub_graph()
    else:
        ei, n = graphs.roman_like(), 22662
    w = _column_costs(ei, n)
    keep = backbone_mask(ei, n, w)
    for var in off:  # "+NAME": on (the pair certificate is off by default), else off
        monkeypatch.setenv(var.lstrip("+"), "1" if var.startswith("+") else "0")
    keep0 = backbone_mask(ei, n, w)
    assert np.array_equal(keep, keep0)
    assert 0 < keep.sum() < len(keep)


@pytest.mark.parametrize("nparts", [2, 3, 4])
def test_backbone_parts_sum_to_whole(gs, nparts):
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    ei, n = graphs.rmat(14, 8, seed=4), 1 << 14
    ip, ix, _ = O.canonical_csr(ei, n)
    w = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")[: ei.shape[1]]
    whole = backbone_mask(ei, n, w)
    parts = [backbone_mask(ei, n, w, part=p, nparts=nparts) for p in range(nparts)]
    tot = np.zeros(len(whole), dtype=int)
    for p in parts:
        tot += p
    assert tot.max() <= 1
    assert np.array_equal(tot.astype(bool), whole)


@pytest.mark.parametrize("metric", ["jaccard", "degree", "approx_er"])
def test_degree_aware_device_equals_reference_walk(gs, metric):
    """Device phases (segment argmax + radix select) vs the reference's loops
    restated on the host (selection.degree_aware_mask), ties included."""
    from gsparse import graphs
    from gsparse.selection import degree_aware_mask, degree_aware_mask_device

    ei, n = graphs.rmat(12, 8, seed=6), 1 << 12
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = gs.GraphSparsifier(data, "cpu")
    if metric == "approx_er":
        sc = sp_._engine.approx_er(epsilon=0.9, blas_threads=1)
    else:
        sc = sp_.compute_scores(metric)
    E = ei.shape[1]
    pick = sp_._engine.segment_argmax(sc, ei[0], n)
    assert (pick == -2).any() or metric == "approx_er"
    for r in [0.05, 0.2, 0.5, 0.8]:
        ref = degree_aware_mask(sc, ei, n, E, r)
        dev = degree_aware_mask_device(sp_._engine, sc, ei, n, E, r)
        assert np.array_equal(ref, dev), (metric, r)


def test_featcos_1433_bow_vs_oracle(gs):
    from gsparse import graphs

    ei = graphs.chung_lu(2708, 5278, seed=0)
    x = graphs.features(2708, 1433, seed=1, kind="bow")
    ip, ix, _ = O.canonical_csr(ei, 2708)
    data = gs.Data(edge_index=torch.from_numpy(ei), x=torch.from_numpy(x), num_nodes=2708)
    sp_ = gs.GraphSparsifier(data, "cpu")
    assert bits_equal(sp_.compute_scores("feature_cosine"), O.feature_cosine(ip, ix, x))
    x64 = x.astype(np.float64)
    assert bits_equal(sp_._engine.feature_cosine(x64), O.feature_cosine(ip, ix, x64))


def test_topk_large_with_ties_and_specials(gs):
    rng = np.random.default_rng(0)
    nnz = 1 << 20
    s = rng.integers(0, 50, nnz).astype(np.float64) / 7.0  # heavy ties
    s[::97] = -0.0
    s[::101] = 0.0
    s[5] = np.inf
    s[6] = -np.inf
    ctx = gs._lib.Context()
    ctx.set_graph_csr(2, np.array([0, 1, 2]), np.array([1, 0], dtype=np.int32), None)
    eng = gs.engine.Engine(ctx)
    for frac in [0.001, 0.3, 0.5, 0.999]:
        for low in (False, True):
            k = int(nnz * frac)
            mask, cut, nb, nt = eng.topk_mask(s, nnz + 5, k, low)
            ref = O.topk_mask(s, nnz + 5, frac, low, kind="stable")
            if int((nnz + 5) * frac) != k:
                ref = np.zeros(nnz + 5, dtype=bool)
                idx = np.argsort(s, kind="stable")
                ref[idx[:k] if low else idx[-k:]] = True
            assert np.array_equal(mask, ref), (frac, low)
            assert mask.sum() == k
    # quirks: num_keep 0 keeps every scored column (idx[-0:]), keep_lowest keeps none
    m0, *_ = eng.topk_mask(s, nnz + 5, 0, False)
    assert m0[:nnz].all() and not m0[nnz:].any()
    m1, *_ = eng.topk_mask(s, nnz + 5, 0, True)
    assert not m1.any()


def test_topk_candidate_paths_vs_stable_argsort(gs, monkeypatch):
    """The 12-bit first pass + candidate selection (default) and the 8-bit passes
    (GSPARSE_TOPK=8) against np.argsort(kind='stable'): scores crowded into one
    12-bit bucket (every candidate pass busy), NaNs, signed zeros, infinities."""
    rng = np.random.default_rng(7)
    nnz = 3 << 18
    crowd = 1.0 + rng.integers(0, 4000, nnz) * 2.0 ** -40  # one 12-bit bucket, many ties
    spread = rng.standard_normal(nnz)
    spread[::1009] = np.nan
    spread[::211] = -0.0
    spread[::223] = 0.0
    spread[7], spread[8] = np.inf, -np.inf
    ctx = gs._lib.Context()
    ctx.set_graph_csr(2, np.array([0, 1, 2]), np.array([1, 0], dtype=np.int32), None)
    eng = gs.engine.Engine(ctx)
    for s in (crowd, spread):
        for mode in (None, "8"):
            if mode:
                monkeypatch.setenv("GSPARSE_TOPK", mode)
            else:
                monkeypatch.delenv("GSPARSE_TOPK", raising=False)
            for frac in (0.01, 0.5, 0.97):
                for low in (False, True):
                    k = int(nnz * frac)
                    mask, cut, nb, nt = eng.topk_mask(s, nnz + 3, k, low)
                    idx = np.argsort(s, kind="stable")
                    ref = np.zeros(nnz + 3, dtype=bool)
                    ref[idx[:k] if low else idx[-k:]] = True
                    assert np.array_equal(mask, ref), (mode, frac, low)
                    sel = s[ref[:nnz]]
                    c = np.nanmax(sel) if low else np.nanmin(sel)
                    if not np.isnan(c):
                        assert cut == c or (cut == 0 and c == 0)
                        beyond = int((s < c).sum()) if low else int(((s > c) | np.isnan(s)).sum())
                        assert nb == beyond and nt == int((s == c).sum()), (mode, frac, low)


def test_edge_cases(gs):
    # isolated nodes, single edge, empty graph, self-loops + duplicates
    for ei, n in [(np.array([[0, 1], [1, 0]]), 5), (np.zeros((2, 0), dtype=np.int64), 3),
                  (np.array([[0, 0, 1, 1, 2, 2], [0, 1, 0, 0, 2, 1]]), 3)]:
        data = gs.Data(edge_index=torch.from_numpy(ei.astype(np.int64)), num_nodes=n)
        sp_ = gs.GraphSparsifier(data, "cpu")
        ip, ix, d = O.canonical_csr(ei, n)
        assert bits_equal(sp_.compute_scores("jaccard"), O.jaccard(ip, ix))
        assert bits_equal(sp_.compute_scores("adamic_adar"), O.adamic_adar(ip, ix))
        assert bits_equal(sp_.compute_scores("degree"), O.degree(ip, ix, d))
        er = sp_._engine.approx_er(blas_threads=1)
        assert bits_equal(er, O.approx_er(ip, ix, d, n, impl="c"))


def test_errors_mirror_reference(gs):
    g = load_golden("karate_test")
    sp_, _ = make(gs, g, with_x=False)
    with pytest.raises(ValueError, match="not supported"):
        sp_.compute_scores("pagerank")
    for bad in (0, -0.1, 1.5):
        with pytest.raises(ValueError, match="retention_ratio"):
            sp_.sparsify("jaccard", bad)
    with pytest.raises(ValueError, match="requires node features"):
        sp_.compute_scores("feature_cosine")
    d, m = sp_.sparsify("jaccard", 1.0, return_mask=True)
    assert m.all() and d.edge_index.shape[1] == 156
    assert sp_.sparsify("jaccard", 0.5).edge_index.size(1) == 78


def test_er_column_split_combines_to_whole(gs):
    """Multi-GPU ApproxER split (pairwise-tree column blocks) is exact on one device."""
    g = load_golden("rmat10")
    sp_, _ = make(gs, g, with_x=False)
    e = sp_._engine
    full = e.approx_er(blas_threads=1)
    k = e.k
    for parts in (2, 4):
        b = gs.engine.er_split(k, parts)
        sums = [e.er_scores(b[i], b[i + 1], finalize=False) for i in range(parts)]
        while len(sums) > 1:
            sums = [sums[i] + sums[i + 1] for i in range(0, len(sums), 2)]
        tot = 0.0 + sums[0]
        tot = np.maximum(np.nan_to_num(tot, nan=1e-10, posinf=1e-10, neginf=1e-10), 1e-10)
        assert bits_equal(tot, full)


# ------------------------------------------------------ device normal stream
@pytest.mark.parametrize("name", SMALL)
def test_approx_er_device_rng_bit_exact(gs, name):
    """R drawn on the device (PCG64 + NumPy's ziggurat) -> identical scores."""
    g = load_golden(name)
    sp_, _ = make(gs, g, with_x=False)
    er = sp_._engine.approx_er(blas_threads=1, rng_mode="device")
    assert bits_equal(er, g["scores_approx_er"])


def test_approx_er_device_rng_roman_full(gs):
    g = load_golden("roman_full")
    sp_, _ = make(gs, g, with_x=False)
    er = sp_._engine.approx_er(blas_threads=1, rng_mode="device")
    assert bits_equal(er, g["scores_approx_er"])


# ---- exact effective resistance (metrics.py:124-175) on fp64 MFMA ----------
@pytest.mark.parametrize("name", exact_er_names())
def test_exact_er_device(gs, name):
    """gs_exact_er vs the reference golden (within the reference's own pinv noise,
    EXACT_ER_ATOL) and vs the lifted oracle (rtol 1e-8: both inverses carry their
    own ~cond(M) * eps rounding; roman2000's path-like components reach 1.1e-9)."""
    import scipy.sparse as sp

    g = load_golden(name)
    n = int(g["num_nodes"])
    adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
    er = gs.calculate_effective_resistance_scores(adj)
    ref = exact_er_golden(name)
    assert er.dtype == np.float64 and er.shape == ref.shape
    assert np.max(np.abs(er - ref), initial=0.0) <= EXACT_ER_ATOL
    lifted = O.exact_er(g["indptr"], g["indices"], g["data"], n, lifted=True)
    np.testing.assert_allclose(er, lifted, rtol=1e-8, atol=1e-12)


def test_exact_er_through_sparsifier(gs):
    g = load_golden("karate_test")
    sp_, _ = make(gs, g, with_x=False)
    er = sp_.compute_scores("effective_resistance")
    assert np.max(np.abs(er - g["scores_effective_resistance"])) <= EXACT_ER_ATOL
    _, m = sp_.sparsify("effective_resistance", 0.5, return_mask=True)
    assert m.dtype == torch.bool and int(m.sum()) > 0


@pytest.mark.parametrize("name", exact_er_names())
def test_exact_er_kept_sets_vs_reference(gs, name):
    """sparsify("effective_resistance", r) kept sets (core.py:229-240) vs the
    reference's own mask of its golden scores: identical for every column whose
    reference score lies outside the reference's pinv noise band (2 x
    EXACT_ER_ATOL) around the cut, and the same kept count; against the lifted
    oracle's scores (the same inverse up to ~cond * eps) the band is 1e-7 relative."""
    import scipy.sparse as sp

    g = load_golden(name)
    n = int(g["num_nodes"])
    ref = exact_er_golden(name)
    E = g["edge_index"].shape[1] if "edge_index" in g else len(ref)
    if "edge_index" in g:
        sp_, _ = make(gs, g, with_x=False)
        got_scores = sp_.compute_scores("effective_resistance")
    else:
        adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
        got_scores = gs.calculate_effective_resistance_scores(adj)
        sp_ = None
    lifted = O.exact_er(g["indptr"], g["indices"], g["data"], n, lifted=True)
    for r in (0.9, 0.6, 0.5, 0.2):
        for low in (False, True):
            k = int(E * r)
            if sp_ is not None:
                _, m = sp_.sparsify("effective_resistance", r, return_mask=True, keep_lowest=low)
                m = m.numpy()
            else:
                m = O.topk_mask(got_scores, E, r, low)
            assert int(m.sum()) == (k if k else (0 if low else len(ref)))  # k == 0: idx[-0:]
            for scores, band in ((ref, 2 * EXACT_ER_ATOL), (lifted, 1e-7 * float(np.max(lifted)))):
                rm = O.topk_mask(scores, E, r, low)
                if k == 0:  # the idx[-0:] quirk: every scored column (top) or none (lowest)
                    assert np.array_equal(m, rm)
                    continue
                srt = np.sort(scores)
                cut = srt[k - 1] if low else srt[len(srt) - k]
                clear = np.abs(scores - cut) > band
                clear = np.concatenate([clear, np.zeros(E - len(scores), dtype=bool)])
                assert np.array_equal(m[clear], rm[clear]), (name, r, low, int((m != rm)[clear].sum()))


@pytest.mark.parametrize("n,blocks", [(3000, 5), (4100, 1), (70, 3)])
def test_exact_er_components_and_padding(gs, n, blocks):
    """Several components (plus isolated nodes), weights, n not a multiple of 64."""
    import scipy.sparse as sp

    rng = np.random.default_rng(n)
    parts = np.array_split(np.arange(n - 3), blocks)
    rows, cols = [], []
    for p in parts:
        m = len(p)
        a = rng.integers(0, m, 4 * m)
        b = rng.integers(0, m, 4 * m)
        keep = a != b
        rows.append(p[a[keep]]), cols.append(p[b[keep]])
        rows.append(p[:-1]), cols.append(p[1:])  # a path keeps each part connected
    r = np.concatenate(rows)
    c = np.concatenate(cols)
    w = rng.uniform(0.5, 2.0, len(r))
    A = sp.coo_matrix((w, (r, c)), shape=(n, n)).tocsr()
    A = (A + A.T).tocsr()
    A.sum_duplicates()
    er = gs.calculate_effective_resistance_scores(A)
    lifted = O.exact_er(A.indptr, A.indices, A.data, n, lifted=True)
    np.testing.assert_allclose(er, lifted, rtol=1e-8, atol=1e-12)


def test_exact_er_rejects_directed(gs):
    import scipy.sparse as sp

    A = sp.csr_matrix(np.array([[0, 1, 0], [0, 0, 1], [1, 0, 0]], dtype=np.float64))
    with pytest.raises(NotImplementedError):
        gs.calculate_effective_resistance_scores(A)
    B = sp.csr_matrix(np.array([[0, 1.0], [2.0, 0]]))
    with pytest.raises(NotImplementedError):
        gs.calculate_effective_resistance_scores(B)


def test_exact_er_empty_graph(gs):
    import scipy.sparse as sp

    er = gs.calculate_effective_resistance_scores(sp.csr_matrix((5, 5)))
    assert er.shape == (0,)


# ---- compute_topology_metrics (metrics.py:445-520), SURVEY 8(f) rank 4 -----
def _topology_cases():
    import scipy.sparse as sp

    out = []
    for name in ["karate_test", "cora_like", "roman2000", "rmat10", "star", "single_edge"]:
        g = load_golden(name)
        n = int(g["num_nodes"])
        out.append((name, sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))))
    # weighted, several components, self-loops, isolated nodes
    rng = np.random.default_rng(7)
    n = 900
    r = rng.integers(0, 600, 2500)
    c = (r + rng.integers(1, 40, 2500)) % 600
    r = np.concatenate([r, np.arange(600, 850), [3, 17, 650]])
    c = np.concatenate([c, np.arange(601, 851) % 850 + (np.arange(600, 850) >= 849) * 600,
                        [3, 17, 650]])
    w = rng.uniform(0.5, 2.0, len(r))
    A = sp.coo_matrix((w, (r, c)), shape=(n, n)).tocsr()
    A = (A + A.T).tocsr()
    A.sum_duplicates()
    out.append(("weighted_components_loops", A))
    # directed, weighted (NetworkX keeps the later stored weight of a pair)
    B = sp.random(300, 300, 0.03, random_state=3, format="csr")
    B.data = rng.uniform(0.5, 2.0, B.nnz)
    out.append(("directed_weighted", B))
    return out


@pytest.mark.parametrize("case", _topology_cases(), ids=lambda c: c[0])
def test_topology_metrics_vs_networkx(gs, case):
    """Exact fields (edges, degrees, clustering, components) identical to the
    reference's NetworkX calls -- the clustering bit for bit; the algebraic
    connectivity within 1e-6 relative (tracemin_lu stops at tol = 1e-8; the
    device value is a Lanczos Ritz value on a Cholesky inverse)."""
    _, adj = case
    ref = O.topology_metrics(adj)
    got = gs.compute_topology_metrics(adj)
    for k in ["num_nodes", "num_edges", "num_connected_components"]:
        assert got[k] == ref[k], k
    for k in ["avg_degree", "clustering_coefficient", "largest_component_ratio"]:
        assert bits_equal(np.array([got[k]]), np.array([ref[k]])), (k, got[k], ref[k])
    np.testing.assert_allclose(got["algebraic_connectivity"], ref["algebraic_connectivity"],
                               rtol=1e-6, atol=1e-14)


def test_topology_preservation_and_counts(gs):
    import scipy.sparse as sp

    g = load_golden("karate_test")
    n = int(g["num_nodes"])
    adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
    sp_, data = make(gs, g, with_x=False)
    sd = sp_.sparsify("jaccard", 0.6)
    ei = sd.edge_index.cpu().numpy()
    sparse = sp.csr_matrix((np.ones(ei.shape[1]), (ei[0], ei[1])), shape=(n, n))
    got = gs.compute_topology_preservation(adj, sparse)
    ref_o, ref_s = O.topology_metrics(adj), O.topology_metrics(sparse)
    assert got["component_change"] == ref_s["num_connected_components"] - ref_o["num_connected_components"]
    assert got["edge_retention"] == ref_s["num_edges"] / ref_o["num_edges"]
    # common-neighbour counts = the Jaccard numerators (A @ A on the 0/1 pattern)
    from gsparse._lib import Context

    ctx = Context()
    ctx.set_graph_csr(n, adj.indptr, adj.indices, adj.data)
    cnt = gs.engine.Engine(ctx).common_neighbors()
    b = (adj > 0).astype(np.float64)
    ref = np.asarray((b @ b)[adj.nonzero()]).ravel()
    assert np.array_equal(cnt, ref)


# ---- sampled-pair shortest paths (compute_geodesic_preservation, verify_geodesic_preservation)
@pytest.mark.parametrize("name", ["karate_test", "cora_like", "roman2000", "rmat10"])
def test_geodesic_analytics_vs_networkx(gs, name):
    """The same sampled pairs, hop distances and weighted Dijkstra distances as the
    reference's NetworkX calls -- equal, not close: every distance is an exact
    left-fold path sum."""
    import scipy.sparse as sp

    g = load_golden(name)
    n = int(g["num_nodes"])
    adj = sp.csr_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, n))
    sp_, data = make(gs, g, with_x=False)
    sd, mask = sp_.sparsify("jaccard", 0.5, return_mask=True)
    ei_s = sd.edge_index.cpu().numpy()
    sparse = sp.csr_matrix((np.ones(ei_s.shape[1]), (ei_s[0], ei_s[1])), shape=(n, n))
    got = gs.compute_geodesic_preservation(adj, sparse, n_samples=300)
    ref = O.geodesic_preservation(adj, sparse, n_samples=300)
    assert got == ref
    # weighted: the metric backbone of the Jaccard costs vs the whole graph
    ei = g["edge_index"]
    cost = g["cost_jaccard"]
    bd, st = gs.compute_metric_backbone(data, cost, epsilon=1e-9, verbose=False)
    keep = st["keep_mask"]
    pairs, dists = O.verify_geodesic(ei, cost, ei[:, keep], cost[keep], n, n_samples=300)
    from gsparse.metric_backbone import pair_distances

    assert len(pairs) == 300
    d_o = pair_distances(ei, n, cost, pairs)
    d_b = pair_distances(ei[:, keep], n, cost[keep], pairs)
    assert np.array_equal(d_o, np.array([a for a, _ in dists]))
    assert np.array_equal(d_b, np.array([b for _, b in dists]))
    from gsparse.metric_backbone import verify_geodesic_preservation

    res = verify_geodesic_preservation(data, bd, cost, cost[keep], n_samples=300)
    assert res["pairs_tested"] == len(pairs) and res["violations"] == 0


@pytest.mark.parametrize("name", ["karate_test", "cora_like", "rmat10"])
def test_geodesic_violations_vs_networkx(gs, name):
    """A subgraph that is NOT the backbone (the top-50% Jaccard mask): the
    violation / unreachable bookkeeping of metric_backbone.py:199-225 on the
    oracle's NetworkX distances."""
    from gsparse.metric_backbone import verify_geodesic_preservation

    g = load_golden(name)
    n = int(g["num_nodes"])
    _, data = make(gs, g, with_x=False)
    ei, cost = g["edge_index"], g["cost_jaccard"]
    keep = g["mask_jaccard_0.5_0"]
    sub = gs.Data(edge_index=torch.from_numpy(ei[:, keep]), num_nodes=n)
    res = verify_geodesic_preservation(data, sub, cost, cost[keep], n_samples=200)
    pairs, dists = O.verify_geodesic(ei, cost, ei[:, keep], cost[keep], n, n_samples=200)
    uo = sum(np.isinf(a) for a, _ in dists)
    ub = sum((not np.isinf(a)) and np.isinf(b) for a, b in dists)
    viol = [abs(a - b) for a, b in dists if not np.isinf(a) and not np.isinf(b) and abs(a - b) > 1e-6]
    assert res["unreachable_original"] == uo and res["unreachable_backbone"] == ub
    assert res["violations"] == len(viol) + ub
    assert res["verified_equal"] == len(pairs) - uo - ub - len(viol)
    if not ub:
        assert res["max_violation"] == (max(viol) if viol else 0.0)
    assert res["violations"] > 0


@pytest.mark.parametrize("threads", ["256", "1024"])
@pytest.mark.parametrize("S", ["2", "4", "8", "16"])
def test_backbone_multi_source_searches(gs, S, threads, monkeypatch):
    """S sources per workgroup (GSPARSE_BB_MULTI, interleaved labels): the keep
    masks of the reference goldens, of the RMAT-12 oracle, and of the
    single-source searches with the certificates off (most columns searched)."""
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    monkeypatch.setenv("GSPARSE_BB_THREADS", threads)
    monkeypatch.setenv("GSPARSE_BB_MULTI", S)
    for name in ["karate_test", "directed_dup", "rmat10", "roman2000", "cora_like", "star"]:
        g = load_golden(name)
        _, data = make(gs, g, with_x=False)
        for m in ["jaccard", "approx_er", "degree"]:
            if f"backbone_{m}_error" in g:
                continue
            _, st = gs.compute_metric_backbone(data, g[f"cost_{m}"], epsilon=1e-9, verbose=False)
            assert np.array_equal(st["keep_mask"], g[f"backbone_{m}"]), (name, m)
    ei, n = graphs.rmat(12, 8, seed=2), 1 << 12
    ip, ix, _ = O.canonical_csr(ei, n)
    cost = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")
    assert np.array_equal(backbone_mask(ei, n, cost[: ei.shape[1]]), O.metric_backbone(ei, n, cost))
    monkeypatch.setenv("GSPARSE_BB_LANDMARKS", "0")
    for ei, n in [(graphs.rmat(14, 8, seed=3), 1 << 14), _hub_graph()]:
        # one weight per column (the hub graph has duplicate columns, so its CSR
        # has fewer entries than edge_index: index the CSR costs by column)
        w = _column_costs(ei, n)
        multi = backbone_mask(ei, n, w)
        monkeypatch.setenv("GSPARSE_BB_MULTI", "1")
        single = backbone_mask(ei, n, w)
        monkeypatch.setenv("GSPARSE_BB_MULTI", S)
        assert np.array_equal(multi, single)


@pytest.mark.parametrize("nearfar", ["0", "0.02", "0.5", "6"])
def test_backbone_near_far_order(gs, nearfar, monkeypatch):
    """k_bb_sssp_multi's near-far order (GSPARSE_BB_NEARFAR = the step as a
    multiple of the median edge weight; 0 = plain frontier order): tiny steps
    (many threshold moves, far piles refilled and compacted often), the default,
    and steps past most distances -- the RMAT-12 oracle's keep mask, and the
    single-source searches' on RMAT-14 / the hub graph with the certificates off."""
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    monkeypatch.setenv("GSPARSE_BB_NEARFAR", nearfar)
    monkeypatch.setenv("GSPARSE_BB_MULTI", "8")
    monkeypatch.setenv("GSPARSE_BB_THREADS", "1024")
    ei, n = graphs.rmat(12, 8, seed=2), 1 << 12
    ip, ix, _ = O.canonical_csr(ei, n)
    cost = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")
    assert np.array_equal(backbone_mask(ei, n, cost[: ei.shape[1]]), O.metric_backbone(ei, n, cost))
    monkeypatch.setenv("GSPARSE_BB_LANDMARKS", "0")
    for ei, n in [(graphs.rmat(14, 8, seed=3), 1 << 14), _hub_graph()]:
        w = _column_costs(ei, n)
        multi = backbone_mask(ei, n, w)
        monkeypatch.setenv("GSPARSE_BB_MULTI", "1")
        single = backbone_mask(ei, n, w)
        monkeypatch.setenv("GSPARSE_BB_MULTI", "8")
        assert np.array_equal(multi, single)


@pytest.mark.parametrize("weights", ["ties", "scales", "asymmetric"])
@pytest.mark.parametrize("order", ["asc", "desc"])
@pytest.mark.parametrize("S", ["8", "16"])
def test_backbone_reverse_columns_vs_oracle(gs, weights, order, S, monkeypatch):
    """The reverse-column decisions of k_bb_sssp_multi (gs_backbone.hip
    bb_cross_decide) on weights that stress their margins: small integers (exact
    ties between an edge and a 2- or 3-edge path, where neither the prune nor the
    exact certificate may fire), costs over 18 decades (fl folds of very different
    magnitudes), and different weights on the two directions of a pair -- 8 (near-far)
    or 16 sources per workgroup in either batch order, against the oracle's per-row Dijkstra
    (metric_backbone.py:86-111), with epsilon 0 and the default."""
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    monkeypatch.setenv("GSPARSE_BB_MULTI", S)  # 8: with the near-far order (default step)
    monkeypatch.setenv("GSPARSE_BB_ORDER", order)
    rng = np.random.default_rng(7)
    ei, n = graphs.rmat(12, 8, seed=5), 1 << 12
    E = ei.shape[1]
    # one weight per undirected pair, then the asymmetric case perturbs one direction
    key = np.minimum(ei[0], ei[1]) * n + np.maximum(ei[0], ei[1])
    _, inv = np.unique(key, return_inverse=True)
    if weights == "ties":
        pw = rng.integers(1, 4, size=inv.max() + 1).astype(np.float64)
    else:
        pw = 10.0 ** rng.uniform(-9, 9, size=inv.max() + 1)
    w = pw[inv]
    if weights == "asymmetric":
        flip = rng.random(E) < 0.3
        w = np.where(flip, w * rng.uniform(0.5, 2.0, size=E), w)
    for eps in (1e-9, 0.0):
        ref = O.metric_backbone(ei, n, w, epsilon=eps)
        assert np.array_equal(backbone_mask(ei, n, w, epsilon=eps), ref), (weights, order, eps)


@pytest.mark.parametrize("weights", ["ties", "scales", "asymmetric"])
def test_backbone_pair_certificate_vs_oracle(gs, weights, monkeypatch):
    """The meet-in-the-middle certificate (k_bb_sssp_multi PAIR, GSPARSE_BB_MITM=1: both
    ends of every open column searched to half its weight, the u-ball's labels plus the
    v-search's labels bounding every alternative path, the direct edge's walks excluded)
    on the margin-stressing weights of the test above, against the oracle's Dijkstra."""
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    monkeypatch.setenv("GSPARSE_BB_MITM", "1")
    rng = np.random.default_rng(11)
    ei, n = graphs.rmat(12, 8, seed=6), 1 << 12
    E = ei.shape[1]
    key = np.minimum(ei[0], ei[1]) * n + np.maximum(ei[0], ei[1])
    _, inv = np.unique(key, return_inverse=True)
    if weights == "ties":
        pw = rng.integers(1, 4, size=inv.max() + 1).astype(np.float64)
    else:
        pw = 10.0 ** rng.uniform(-9, 9, size=inv.max() + 1)
    w = pw[inv]
    if weights == "asymmetric":
        flip = rng.random(E) < 0.3
        w = np.where(flip, w * rng.uniform(0.5, 2.0, size=E), w)
    for eps in (1e-9, 0.0):
        ref = O.metric_backbone(ei, n, w, epsilon=eps)
        assert np.array_equal(backbone_mask(ei, n, w, epsilon=eps), ref), (weights, eps)
