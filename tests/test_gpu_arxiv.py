"""configs[2] at full size: the ogbn-arxiv stand-in (gsparse.graphs.citation_like,
n = 169,343, symmetrised, ~2.3M CSR entries).

* Jaccard over every entry, bit-exact vs the oracle (metrics.py:17-64).
* ApproxER (metrics.py:178-298) at k = 3,210: every n x k device buffer is
  4.4 GB, so the 64-bit offset paths of the projection, the CG and the
  per-edge sums are exercised.  JL columns [0, 16) and [k-16, k) are solved on
  the device and compared bit for bit with the oracle's CG (T = 8 BLAS chunks)
  on the same columns of Y = B @ R, the oracle streaming R = N(0,1)^{m x k}
  from NumPy's PCG64 in row chunks and keeping those columns only.
"""

import numpy as np
import pytest
import scipy.sparse as sp
import torch

import gsparse_oracle as O
from conftest import bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def arxiv():
    from gsparse import graphs

    ei = graphs.citation_like()
    n = 169_343
    ip, ix, d = O.canonical_csr(ei, n)
    return ei, n, ip, ix, d


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


def test_arxiv_jaccard_bit_exact(gs, arxiv):
    ei, n, ip, ix, _ = arxiv
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    assert np.array_equal(sp_.adj.indptr, ip) and np.array_equal(sp_.adj.indices, ix)
    assert bits_equal(sp_.compute_scores("jaccard"), O.jaccard(ip, ix))


def _y_columns(ip, ix, n, k, cols, seed=42, rows_per_chunk=8192):
    """Y[:, cols] of metrics.py:260-275 with R streamed in row chunks (the
    NumPy stream is chunk-invariant)."""
    rows = O.csr_rows(ip)
    mask = rows < ix
    u_e, v_e = rows[mask], ix[mask].astype(np.int64)
    m = len(u_e)
    rng = np.random.default_rng(seed)
    Rc = np.empty((m, len(cols)), dtype=np.float64)
    for e0 in range(0, m, rows_per_chunk):
        e1 = min(m, e0 + rows_per_chunk)
        Rc[e0:e1] = rng.standard_normal((e1 - e0, k))[:, cols]
    Rc /= np.sqrt(k)
    B = sp.csr_matrix((np.concatenate([np.ones(m), -np.ones(m)]),
                       (np.concatenate([u_e, v_e]), np.concatenate([np.arange(m), np.arange(m)]))),
                      shape=(n, m))
    return B @ Rc


@pytest.mark.timeout(900)
def test_arxiv_approx_er_column_blocks(gs, arxiv):
    ei, n, ip, ix, d = arxiv
    k = O.jl_dim(n)
    assert k == 3210
    cols = list(range(16)) + list(range(k - 16, k))
    Y = _y_columns(ip, ix, n, k, cols)
    L = O.laplacian_reg(ip, ix, d, n)
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    e = sp_._engine
    e.er_prepare(k)
    e.er_project_device(np.random.default_rng(42), k)
    for j, (c0, c1) in enumerate(((0, 16), (k - 16, k))):
        Z, its = O.cg(L, np.ascontiguousarray(Y[:, 16 * j:16 * (j + 1)]), 500, 1e-6, 8)
        assert its.max() <= 500
        e.er_solve(c0, c1, 500, 1e-6, 8)
        got = e.er_scores(c0, c1, finalize=False)
        ref = O.er_from_z(ip, ix, Z)
        # er_from_z clamps at 1e-10 as metrics.py:296-297; the partial sums are far above it
        assert np.all(ref > 1e-10)
        assert bits_equal(got, ref), (c0, float(np.max(np.abs(got - ref) / ref)))
