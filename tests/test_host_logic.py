"""Host logic of the drop-in API that needs no GPU.

Metric-name normalisation, the cost transform, the NumPy-defined selection
helpers (sampled / degree-aware), the Data stand-in, the synthetic graph
generators, the JL dimension and the Adamic-Adar weight table -- each
checked against the reference's golden vectors or its documented answers.
"""

import os

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import ROOT, golden_names, load_golden
from gsparse import graphs
from gsparse.core import GraphSparsifier
from gsparse.data import Data
from gsparse.engine import aa_weights, jl_dim
from gsparse.selection import degree_aware_mask, numpy_topk_mask, sampled_mask

SMALL = golden_names(include_big=False)


def bare_sparsifier():
    return GraphSparsifier.__new__(GraphSparsifier)


def test_normalize_metric_names():
    s = bare_sparsifier()
    cases = {"jaccard": "jaccard", "Adamic-Adar": "adamic_adar", "aa": "adamic_adar",
             "ER": "effective_resistance", "effective-resistance": "effective_resistance",
             "approx_er": "approx_effective_resistance", "rand": "random",
             "degree": "degree", "Feature Cosine": "feature_cosine",
             "feature-cosine": "feature_cosine"}
    for k, v in cases.items():
        assert s._normalize_metric_name(k) == v
    with pytest.raises(ValueError, match="not supported"):
        s._normalize_metric_name("pagerank")


def test_scores_to_cost_known_answer():
    # tests/test_sparsification.py:143-150
    s = bare_sparsifier()
    np.testing.assert_allclose(s._scores_to_cost(np.array([0.5, 1.0, 0.25]), "jaccard"),
                               [1.0, 0.0, 3.0])
    assert np.all(s._scores_to_cost(np.zeros(4), "jaccard") == 1.0)


@pytest.mark.parametrize("name", SMALL)
def test_scores_to_cost_matches_golden(name):
    g = load_golden(name)
    s = bare_sparsifier()
    for m in ["jaccard", "adamic_adar", "degree", "approx_er"]:
        c = s._scores_to_cost(g[f"scores_{m}"], m)
        assert np.array_equal(c.view(np.uint64), g[f"cost_{m}"].view(np.uint64))


@pytest.mark.parametrize("name", SMALL)
def test_sampled_and_degree_aware_match_golden(name):
    g = load_golden(name)
    E = g["edge_index"].shape[1]
    n = int(g["num_nodes"])
    for m in ["jaccard", "adamic_adar", "degree", "approx_er", "feature_cosine"]:
        if f"scores_{m}" not in g:
            continue
        s = g[f"scores_{m}"]
        for r in (0.5, 0.2):
            if f"sampled_{m}_{r}" in g:
                assert np.array_equal(sampled_mask(s, E, r, 42), g[f"sampled_{m}_{r}"])
            elif f"sampled_{m}_{r}_error" in g:
                with pytest.raises(ValueError):
                    sampled_mask(s, E, r, 42)
            if f"degaware_{m}_{r}" in g:
                got = degree_aware_mask(s, g["edge_index"], n, E, r)
                assert np.array_equal(got, g[f"degaware_{m}_{r}"]), (m, r)
            elif f"degaware_{m}_{r}_error" in g:
                with pytest.raises(IndexError):
                    degree_aware_mask(s, g["edge_index"], n, E, r)


@pytest.mark.parametrize("name", SMALL)
def test_numpy_topk_mask_is_reference(name):
    g = load_golden(name)
    E = g["edge_index"].shape[1]
    for r in [0.9, 0.5, 0.2]:
        for low in (0, 1):
            got = numpy_topk_mask(g["scores_jaccard"], E, int(E * r), bool(low))
            assert np.array_equal(got, g[f"mask_jaccard_{r}_{low}"])


def test_aa_weights_and_jl_dim():
    g = load_golden("rmat10")
    assert np.array_equal(aa_weights(g["indptr"]), O.aa_weights(g["indptr"]))
    assert jl_dim(22662, 0.3) == 2674
    assert jl_dim(2708, 0.3) == 2107
    assert jl_dim(1, 0.3) == jl_dim(2, 0.3)
    assert jl_dim(169343, 0.3) == 3210


def test_data_standin():
    ei = torch.tensor([[0, 1], [1, 0]])
    d = Data(edge_index=ei, num_nodes=3, y=torch.zeros(3))
    assert d.num_nodes == 3
    c = d.clone()
    c.edge_index[0, 0] = 7
    assert d.edge_index[0, 0] == 0
    assert d.to("cpu").y.shape == (3,)
    assert Data(edge_index=ei).num_nodes == 2


def test_generators_are_deterministic_and_canonical():
    a = graphs.roman_like(2000, 2906, seed=3)
    b = graphs.roman_like(2000, 2906, seed=3)
    assert np.array_equal(a, b)
    assert a.shape == (2, 2 * 2906)
    keys = a[0] * 2000 + a[1]
    assert np.all(np.diff(keys) > 0)  # row-major sorted, duplicate free
    rev = np.sort(a[1] * 2000 + a[0])
    assert np.array_equal(np.sort(keys), rev)  # symmetric
    r = graphs.rmat(10, 16, seed=1)
    assert np.array_equal(r, load_golden("rmat10")["edge_index"])
    full = graphs.roman_like()
    assert full.shape == (2, 65854)


def test_short_edge_weights_raise_index_error():
    """metric_backbone.py:73-74 reads edge_weights[idx] for every column: fewer
    weights than columns is an IndexError before anything reaches libgsparse
    (host-only checks; the library re-checks the count it is given)."""
    from gsparse.distributed import sharded_backbone
    from gsparse.metric_backbone import check_weights

    check_weights(np.zeros(5), 5)
    check_weights(np.zeros(6), 5)
    with pytest.raises(IndexError):
        check_weights(np.zeros(4), 5)
    ei = np.array([[0, 1, 1, 2], [1, 0, 2, 1]])
    with pytest.raises(IndexError):
        sharded_backbone(None, ei, 3, np.ones(3), stages=object())


def test_default_device_follows_torch_current_device(monkeypatch):
    """roman_empire_gpu.py:209-213: torch.cuda.set_device(k) then
    GraphSparsifier(data, device='cpu') -- the context goes to k.  Order:
    $GSPARSE_DEVICE, torch's current device once CUDA is initialised,
    $LOCAL_RANK, 0.  (Host logic only; the GPU test does it for real.)"""
    import torch

    from gsparse import _lib

    monkeypatch.delenv("GSPARSE_DEVICE", raising=False)
    monkeypatch.delenv("LOCAL_RANK", raising=False)
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: False)
    assert _lib.default_device() == 0
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    assert _lib.default_device() == 3
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert _lib.default_device() == 3  # the caller's set_device wins over the launcher's rank
    monkeypatch.setenv("GSPARSE_DEVICE", "2")
    assert _lib.default_device() == 2


def test_blas_threads_default_is_openblas_count():
    """The drop-in reproduces the calling process's OpenBLAS thread count."""
    from threadpoolctl import threadpool_limits

    from gsparse.engine import blas_threads_default

    for t in (1, 3, 16, 64):
        with threadpool_limits(limits=t, user_api="blas"):
            assert blas_threads_default() == t


def test_blas_threads_default_clamped_to_openblas_max(monkeypatch):
    """OpenBLAS runs at most MAX_THREADS (64) threads whatever is asked for."""
    from gsparse.engine import blas_threads_default

    monkeypatch.setenv("GSPARSE_BLAS_THREADS", "200")
    assert blas_threads_default() == 64
    monkeypatch.setenv("GSPARSE_BLAS_THREADS", "7")
    assert blas_threads_default() == 7


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N starts N ranks itself, and fails loudly when fewer
    than N GPUs are visible (none here)."""
    import subprocess
    import sys

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--steps", "1"], capture_output=True, text=True, timeout=300,
                       env={k: v for k, v in os.environ.items()
                            if k not in ("WORLD_SIZE", "GSPARSE_REHEARSE")})
    assert r.returncode != 0
    assert "needs 2 GPUs" in (r.stderr + r.stdout)


def test_backbone_phases_cut_the_batch_list(monkeypatch):
    """gsparse.distributed.backbone_phases: one range on one rank; the default cuts at
    BB_PHASES (BB_PHASES_4 at 4-7 ranks) of the batch list; $GSPARSE_BB_PHASES and an
    explicit list override them; the ranges tile [0, nbatch) in order."""
    from gsparse.distributed import BB_PHASES, BB_PHASES_4, backbone_phases

    monkeypatch.delenv("GSPARSE_BB_PHASES", raising=False)
    assert backbone_phases(1000, 1) == [(0, 1000)]
    assert backbone_phases(0, 8) == [(0, 0)]
    for world, fr in ((2, BB_PHASES), (3, BB_PHASES), (4, BB_PHASES_4), (7, BB_PHASES_4), (8, BB_PHASES)):
        rng = backbone_phases(1000, world)
        assert [b for _, b in rng[:-1]] == [int(round(f * 1000)) for f in fr]
        assert rng[0][0] == 0 and rng[-1][1] == 1000
        assert all(a1 == b0 for (_, a1), (b0, _) in zip(rng, rng[1:]))
    assert backbone_phases(1000, 8, []) == [(0, 1000)]
    assert backbone_phases(1000, 8, [0.25, 0.5]) == [(0, 250), (250, 500), (500, 1000)]
    monkeypatch.setenv("GSPARSE_BB_PHASES", "0.5")
    assert backbone_phases(1000, 2) == [(0, 500), (500, 1000)]


def test_counter_join_skips_first_call_kernels():
    """bench.kernel_counters: the profiled run has one call of the region; the Jaccard
    plan kernels (launched by the first call on a graph only) are left out of the per-call
    counters joined to the timed steps, and named."""
    import importlib.util
    import os

    root = os.path.join(os.path.dirname(__file__), "..")
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    summ = {"_meta": {"calls_per_run": 1},
            "gs::k_jac_plan(long const*)": {"launches": 1, "FETCH_SIZE_KB_per_launch": 100.0,
                                            "WRITE_SIZE_KB_per_launch": 10.0},
            "void gs::k_jac_hashq<32768, 1024, 8>(long const*)": {
                "launches": 2, "FETCH_SIZE_KB_per_launch": 7.0, "WRITE_SIZE_KB_per_launch": 1.0},
            "gs::k_bb_keep(long const*)": {"launches": 1, "FETCH_SIZE_KB_per_launch": 5.0,
                                          "WRITE_SIZE_KB_per_launch": 5.0}}
    c = b.kernel_counters(summ, "jaccard", 1.0)
    assert c["FETCH_SIZE_KB"] == 14.0 and c["WRITE_SIZE_KB"] == 2.0 and c["kernels"] == 1
    assert c["first_call_only"] == ["gs::k_jac_plan"]
    bb = b.kernel_counters(summ, "metric_backbone", 1.0)
    assert bb["FETCH_SIZE_KB"] == 5.0 and bb["first_call_only"] == []


def test_citation_like_rejects_impossible_counts():
    """more distinct citations than n (n - 1) / 2 pairs raise instead of
    looping; the limit itself is reachable."""
    from gsparse import graphs

    with pytest.raises(ValueError):
        graphs.citation_like(5, 11)
    with pytest.raises(ValueError):
        graphs.citation_like(1, 0)
    assert graphs.citation_like(5, 10).shape == (2, 20)
