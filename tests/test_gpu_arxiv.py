"""configs[2] at full size: the ogbn-arxiv stand-in (gsparse.graphs.citation_like,
n = 169,343, symmetrised, ~2.3M CSR entries).

* Jaccard over every entry, bit-exact vs the oracle (metrics.py:17-64).
* ApproxER (metrics.py:178-298) at k = 3,210: every n x k device buffer is
  4.4 GB, so the 64-bit offset paths of the projection, the CG and the
  per-edge sums are exercised.  JL columns [0, 16) and [k-16, k) are solved on
  the device and compared bit for bit with the oracle's CG (T = 8 BLAS chunks)
  on the same columns of Y = B @ R, the oracle streaming R = N(0,1)^{m x k}
  from NumPy's PCG64 in row chunks and keeping those columns only.
* The timed geometry (bench.py --workload arxiv): all k columns solved in one
  er_solve -- 128-column blocks through the batched kernels -- then the whole
  block [1536, 1664) and the tail [k-16, k) read back with er_z and compared bit
  for bit with the oracle's CG on the same Y columns.
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


K_ARXIV = 3210
BLOCK = (1536, 1664)  # a whole 128-column block of the full solve


@pytest.fixture(scope="module")
def arxiv_y(arxiv):
    """Y columns [0, 16), [k-16, k) and BLOCK from one pass over the R stream."""
    ei, n, ip, ix, d = arxiv
    k = O.jl_dim(n)
    assert k == K_ARXIV
    cols = list(range(16)) + list(range(k - 16, k)) + list(range(*BLOCK))
    return _y_columns(ip, ix, n, k, cols)


def test_arxiv_stand_in_size(arxiv):
    """SURVEY 8(d) configs[2]: ogbn-arxiv's 1,166,243 citations, one per undirected pair."""
    ei, n, ip, ix, _ = arxiv
    assert n == 169_343 and ei.shape[1] == 2 * 1_166_243 == len(ix)
    assert int(np.count_nonzero(ei[0] < ei[1])) == 1_166_243


@pytest.mark.timeout(900)
def test_arxiv_approx_er_column_blocks(gs, arxiv, arxiv_y):
    ei, n, ip, ix, d = arxiv
    k = O.jl_dim(n)
    Y = arxiv_y
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


@pytest.mark.timeout(900)
def test_arxiv_full_solve_block_pin(gs, arxiv, arxiv_y):
    """The bench's geometry: every column in one er_solve (128-column blocks of the
    batched CG), then a whole block and the last 16 columns read back (er_z) and
    compared bit for bit with the oracle CG on the same Y columns (metrics.py:284-289)."""
    ei, n, ip, ix, d = arxiv
    k = O.jl_dim(n)
    L = O.laplacian_reg(ip, ix, d, n)
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    e = sp_._engine
    e.er_prepare(k)
    e.er_project_device(np.random.default_rng(42), k)
    e.er_solve(0, k, 500, 1e-6, 8)
    its_dev = e.er_iterations()
    from test_gpu_pins import _oracle_cg_columns

    for (c0, c1), y0 in ((BLOCK, 32), ((k - 16, k), 16)):
        Z, its = _oracle_cg_columns(L, arxiv_y, list(range(y0, y0 + c1 - c0)))
        assert np.array_equal(its_dev[c0:c1], its), (c0, its_dev[c0:c1], its)
        got = e.er_z(c0, c1)
        assert bits_equal(got, Z), (c0, float(np.max(np.abs(got - Z))))
