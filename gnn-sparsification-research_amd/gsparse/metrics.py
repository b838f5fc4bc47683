"""Edge metrics -- drop-in for ``src/sparsification/metrics.py``.

Same names, signatures, defaults and return contract (float64 array in the
order of ``adj.nonzero()``) as the reference; the arithmetic runs in
libgsparse.so on the MI355X.  Inputs must be SciPy sparse matrices with
non-negative entries and no duplicate entries (canonical CSR, the form every
reference caller builds); unsorted rows are accepted and mapped back to
storage order.
"""

from __future__ import annotations

import threading
from typing import Dict

import numpy as np
import scipy.sparse as sp
from numpy.typing import NDArray

from ._lib import Context
from .engine import Engine

_CTX = {}
_CTX_LOCK = threading.Lock()


def _scratch_context() -> Context:
    """One cached context per (thread, device) for the module-level functions."""
    key = (threading.get_ident(),)
    with _CTX_LOCK:
        ctx = _CTX.get(key)
        if ctx is None:
            ctx = Context()
            _CTX[key] = ctx
        return ctx


def _prepare(adj):
    """-> (csr canonical copy or view, perm) where perm maps canonical -> storage order."""
    if not sp.issparse(adj):
        adj = sp.csr_matrix(np.asarray(adj))
    a = sp.csr_matrix(adj)
    if a.shape[0] != a.shape[1]:
        raise ValueError(f"adjacency must be square, got {a.shape}")
    data = np.asarray(a.data)
    if np.any(data < 0):
        raise NotImplementedError("negative adjacency entries are outside the supported contract")
    if np.any(data == 0):
        a = a.copy()
        a.eliminate_zeros()
    perm = None
    if not a.has_canonical_format:
        n = a.shape[0]
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(a.indptr))
        keys = rows * n + a.indices.astype(np.int64)
        order = np.argsort(keys, kind="stable")
        if np.any(keys[order][1:] == keys[order][:-1]):
            raise NotImplementedError("duplicate entries in adj (call adj.sum_duplicates())")
        perm = order  # canonical position p holds storage entry order[p]
        a = sp.csr_matrix((a.data[order], a.indices[order], a.indptr), shape=a.shape)
    return a, perm


def _engine(adj):
    a, perm = _prepare(adj)
    ctx = _scratch_context()
    ctx.set_graph_csr(a.shape[0], a.indptr, a.indices, a.data)
    return Engine(ctx), perm


def _unpermute(scores, perm):
    if perm is None:
        return scores
    out = np.empty_like(scores)
    out[perm] = scores
    return out


def calculate_jaccard_scores(adj: sp.csr_matrix) -> NDArray[np.float64]:
    """Jaccard J(u,v) = |N(u) ∩ N(v)| / |N(u) ∪ N(v)| for every edge (metrics.py:17-64).

    Bit-identical to the reference: integer intersection counts, one fp64
    divide, 0 when the union is empty."""
    eng, perm = _engine(adj)
    return _unpermute(eng.jaccard(), perm)


def calculate_adamic_adar_scores(adj: sp.csr_matrix) -> NDArray[np.float64]:
    """Adamic-Adar with log(deg+1) weights (metrics.py:67-121), bit-identical."""
    eng, perm = _engine(adj)
    return _unpermute(eng.adamic_adar(), perm)


def calculate_effective_resistance_scores(adj: sp.csr_matrix) -> NDArray[np.float64]:
    """EXACT effective resistance (metrics.py:124-175), dense, on the MI355X.

    The reference reads R(u,v) = P_uu + P_vv - 2 P_uv off pinv(L + 1e-10 I); this
    reads it off inv(L + sum_C J_C/|C|) (equal in exact arithmetic for every
    edge, whose endpoints share a component), inverted by Newton-Schulz on fp64
    MFMA (gs_exact_er).  Agrees with the reference to its own pinv rounding
    noise (<= 1e-4 relative on the fixtures; DESIGN.md §Exact ER).  Symmetric
    adjacency with n <= 32768 only (NotImplementedError otherwise)."""
    eng, perm = _engine(adj)
    return _unpermute(eng.exact_er(), perm)


def calculate_approx_effective_resistance_scores(
    adj: sp.csr_matrix,
    epsilon: float = 0.3,
    seed: int = 42,
    max_cg_iters: int = 500,
    cg_tol: float = 1e-6,
) -> NDArray[np.float64]:
    """Spielman-Srivastava JL-sketched effective resistance (metrics.py:178-298).

    Same JL dimension, PCG64 normal stream, incidence projection, SciPy-1.15
    CG recurrence and OpenBLAS ddot reduction order as the reference, batched
    over all k columns on the GPU."""
    eng, perm = _engine(adj)
    return _unpermute(eng.approx_er(epsilon, seed, max_cg_iters, cg_tol), perm)


def calculate_feature_cosine_scores(adj: sp.csr_matrix, features: np.ndarray) -> NDArray[np.float64]:
    """Cosine similarity of L2-normalised node features per edge (metrics.py:301-358).

    Computed in the features' dtype with NumPy's pairwise summation order,
    clamped at 0, returned as float64 -- bit-identical."""
    eng, perm = _engine(adj)
    return _unpermute(eng.feature_cosine(features), perm)


def compute_geodesic_preservation(
    original_adj: sp.csr_matrix,
    sparse_adj: sp.csr_matrix,
    n_samples: int = 500,
    seed: int = 42,
) -> Dict:
    """Geodesic (hop-distance) preservation between sampled node pairs
    (metrics.py:361-442): the reference's RNG calls and bookkeeping, the hop
    distances of ``nx.from_scipy_sparse_array``'s graphs from gs_pair_distances
    (exact, unit weights)."""
    from .metric_backbone import pair_distances

    n = original_adj.shape[0]
    rng = np.random.default_rng(seed)
    pairs = set()
    max_attempts = n_samples * 10
    attempts = 0
    while len(pairs) < n_samples and attempts < max_attempts:
        u, v = rng.integers(0, n, size=2)
        if u != v:
            pairs.add((min(u, v), max(u, v)))
        attempts += 1
    pairs = list(pairs)

    def hops(adj):
        coo = sp.coo_matrix(adj)
        r = coo.row.astype(np.int64)
        c = coo.col.astype(np.int64)
        ei = np.stack([np.concatenate([r, c]), np.concatenate([c, r])])
        return pair_distances(ei, adj.shape[0], None, pairs) if pairs else np.zeros(0)

    d_o, d_s = hops(original_adj), hops(sparse_adj)
    preserved = 0
    increased = 0
    disconnected = 0
    distance_increases = []
    for a, b in zip(d_o, d_s):
        if np.isinf(a):
            continue  # already disconnected in the original
        if np.isinf(b):
            disconnected += 1
            continue
        d_orig, d_sparse = int(a), int(b)
        if d_sparse == d_orig:
            preserved += 1
        else:
            increased += 1
            distance_increases.append(d_sparse - d_orig)
    total_valid = preserved + increased + disconnected
    preservation_ratio = preserved / total_valid if total_valid > 0 else 0.0
    return {
        "preservation_ratio": preservation_ratio,
        "pairs_tested": len(pairs),
        "preserved_count": preserved,
        "increased_count": increased,
        "disconnected_count": disconnected,
        "avg_distance_increase": np.mean(distance_increases) if distance_increases else 0.0,
        "max_distance_increase": max(distance_increases) if distance_increases else 0,
    }


def _nx_graph_arrays(adj):
    """The graph nx.from_scipy_sparse_array(adj) builds (metrics.py:464): one
    undirected edge per stored entry (u, v), self-loops kept.  -> (symmetric
    self-loop-free 0/1 pattern S, bool[n] self-loop flags, weighted symmetric
    copy W of the off-diagonal weights as NetworkX keeps them, or None when a
    kept weight is not positive)."""
    a = sp.csr_matrix(adj)
    n = a.shape[0]
    if a.shape[0] != a.shape[1]:
        raise ValueError(f"adjacency must be square, got {a.shape}")
    coo = a.tocoo()
    r = coo.row.astype(np.int64)
    c = coo.col.astype(np.int64)
    loops = np.zeros(n, dtype=bool)
    loops[r[r == c]] = True
    off = r != c
    u = np.concatenate([r[off], c[off]])
    v = np.concatenate([c[off], r[off]])
    S = sp.csr_matrix((np.ones(len(u)), (u, v)), shape=(n, n))
    S.sum_duplicates()
    S.data[:] = 1.0
    S.sort_indices()
    # the weight of edge {u, v}: NetworkX adds the stored entries in CSR order, so
    # the later one wins -- (max, min) over (min, max) when both are stored
    d = coo.data.astype(np.float64)
    lo, up = r > c, r < c
    keys = np.concatenate([c[up] * n + r[up], r[lo] * n + c[lo]])
    vals = np.concatenate([d[up], d[lo]])
    order = np.argsort(keys, kind="stable")
    ks, vs = keys[order], vals[order]
    last = np.r_[ks[1:] != ks[:-1], True] if len(ks) else np.zeros(0, dtype=bool)
    ks, vs = ks[last], vs[last]
    hi_, lo_ = ks // max(n, 1), ks % max(n, 1)
    Wt = sp.csr_matrix((np.concatenate([vs, vs]), (np.concatenate([hi_, lo_]),
                                                    np.concatenate([lo_, hi_]))), shape=(n, n))
    Wt.sort_indices()
    ok = bool(np.all(vs > 0)) and Wt.nnz == S.nnz
    return S, loops, (Wt if ok else None)


def _fiedler(W: sp.csr_matrix) -> float:
    ctx = _scratch_context()
    W = sp.csr_matrix(W)
    W.sort_indices()
    ctx.set_graph_csr(W.shape[0], W.indptr, W.indices, W.data)
    return Engine(ctx).fiedler()


def compute_topology_metrics(adj: sp.csr_matrix) -> Dict:
    """Topological metrics of a graph (metrics.py:445-520) on the device.

    The graph is the one ``nx.from_scipy_sparse_array(adj)`` builds.  Edge count,
    degrees, clustering (``gs_clustering``, NetworkX's exact operation order) and
    components (``gs_components``) are exact; the algebraic connectivity of the
    graph (or of its largest component) is ``gs_fiedler`` -- 1 / lambda_max of the
    Laplacian pseudo-inverse, Lanczos on an fp64-MFMA Cholesky inverse -- to
    ~1e-10 relative where the reference's tracemin_lu stops at tol = 1e-8.
    Dense: the largest component must have <= 32768 nodes."""
    n = adj.shape[0]
    S, loops, W = _nx_graph_arrays(adj)
    num_edges = int(S.nnz // 2 + np.count_nonzero(loops))
    degrees = np.diff(S.indptr).astype(np.int64) + 2 * loops.astype(np.int64)
    avg_degree = degrees.mean() if len(degrees) > 0 else 0.0
    ctx = _scratch_context()
    ctx.set_graph_csr(n, S.indptr, S.indices, S.data)
    eng = Engine(ctx)
    clustering = eng.clustering() if n > 0 else 0.0
    labels, num_components, largest = eng.components() if n > 0 else (np.zeros(0), 0, 0)
    largest_component_ratio = largest / n if n > 0 else 0.0
    algebraic_connectivity = 0.0
    if num_components >= 1 and n > 1:
        if num_components == 1:
            nodes = None
        else:
            # max(components, key=len): the first largest in discovery order, i.e. the
            # one with the smallest node id among the largest
            roots, sizes = np.unique(labels, return_counts=True)
            root = roots[np.argmax(sizes)]
            nodes = np.flatnonzero(labels == root)
        if nodes is None or len(nodes) > 1:
            if W is None:
                raise NotImplementedError("algebraic connectivity of an adjacency with zero or "
                                          "negative edge weights")
            sub = W if nodes is None else W[nodes][:, nodes]
            algebraic_connectivity = _fiedler(sub)
    return {
        "num_nodes": n,
        "num_edges": num_edges,
        "avg_degree": avg_degree,
        "clustering_coefficient": clustering,
        "algebraic_connectivity": algebraic_connectivity,
        "num_connected_components": int(num_components),
        "largest_component_ratio": largest_component_ratio,
    }


def compute_topology_preservation(original_adj: sp.csr_matrix, sparse_adj: sp.csr_matrix) -> Dict:
    """How well topology is preserved after sparsification (metrics.py:523-575)."""
    orig_metrics = compute_topology_metrics(original_adj)
    sparse_metrics = compute_topology_metrics(sparse_adj)
    edge_retention = (sparse_metrics["num_edges"] / orig_metrics["num_edges"]
                      if orig_metrics["num_edges"] > 0 else 0.0)
    clustering_preservation = (
        sparse_metrics["clustering_coefficient"] / orig_metrics["clustering_coefficient"]
        if orig_metrics["clustering_coefficient"] > 0 else 1.0)
    connectivity_preservation = (
        sparse_metrics["algebraic_connectivity"] / orig_metrics["algebraic_connectivity"]
        if orig_metrics["algebraic_connectivity"] > 0 else 0.0)
    component_change = (sparse_metrics["num_connected_components"]
                        - orig_metrics["num_connected_components"])
    return {
        "edge_retention": edge_retention,
        "clustering_preservation": clustering_preservation,
        "connectivity_preservation": connectivity_preservation,
        "component_change": component_change,
        "original_metrics": orig_metrics,
        "sparse_metrics": sparse_metrics,
    }
