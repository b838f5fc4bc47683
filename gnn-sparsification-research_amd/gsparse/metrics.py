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


def compute_geodesic_preservation(*args, **kwargs):  # pragma: no cover - analysis helper
    raise NotImplementedError("NetworkX geodesic analysis is outside the accelerated path "
                              "(SURVEY §8(f)); use the reference implementation")


def compute_topology_metrics(*args, **kwargs):  # pragma: no cover
    raise NotImplementedError("topology analytics are outside the accelerated path (SURVEY §8(f))")


def compute_topology_preservation(*args, **kwargs):  # pragma: no cover
    raise NotImplementedError("topology analytics are outside the accelerated path (SURVEY §8(f))")
