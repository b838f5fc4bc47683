"""ApproxER at the BLAS thread counts the drop-in really meets.

The reference's CG dot products are OpenBLAS ddot calls whose reduction order
follows OpenBLAS's thread count (metrics.py:284-289; n > 10000 splits a dot
into T thread chunks).  GraphSparsifier reproduces the count of the calling
process (gsparse.engine.blas_threads_default: threadpoolctl's OpenBLAS
threads -- 16 on the GPU box, where OPENBLAS_NUM_THREADS=16; at most 64, the
MAX_THREADS of NumPy's OpenBLAS build).  Pinned here at T = 16, 32, 64 and the
process default, against the oracle's restated order (itself pinned to np.dot
at those counts in tests/test_oracle_golden.py), at n = 12,000 in every CG
mode and at configs[1] size (n = 22,662) for JL column blocks of 16.
"""

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal, load_golden

pytestmark = pytest.mark.gpu

THREADS = [16, 32, 64]


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


@pytest.fixture(scope="module")
def chunked_hi():
    from gsparse import graphs

    n = 12000
    ei = graphs.roman_like(n, 17500, seed=3)
    ip, ix, d = O.canonical_csr(ei, n)
    ref = {t: O.approx_er(ip, ix, d, n, epsilon=0.9, max_cg_iters=60, impl="c", blas_threads=t)
           for t in THREADS}
    return n, ei, ref


@pytest.mark.parametrize("mode", ["auto", "0", "1", "3", "4", "5"])
@pytest.mark.parametrize("threads", THREADS)
def test_approx_er_high_blas_threads(gs, chunked_hi, threads, mode, monkeypatch):
    """T = 16 (the box's default), 32 and 64 thread chunks in every CG mode (5
    needs 32 T <= 512 chains and falls back to the resident solver above T = 16)."""
    if mode != "auto":
        monkeypatch.setenv("GSPARSE_CG_MODE", mode)
    n, ei, ref = chunked_hi
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    er = sp_._engine.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=threads)
    assert bits_equal(er, ref[threads])


def test_more_than_64_blas_threads_run_as_64(gs, chunked_hi):
    """OpenBLAS caps its thread count at MAX_THREADS (64): a larger request orders the
    ddot sums as 64 threads do -- here as in the library (gs_er_solve clamps)."""
    n, ei, ref = chunked_hi
    sp_ = gs.GraphSparsifier(gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n), "cpu")
    assert bits_equal(sp_._engine.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=65), ref[64])
    assert bits_equal(sp_._engine.approx_er(epsilon=0.9, max_cg_iters=60, blas_threads=200), ref[64])


@pytest.fixture(scope="module")
def roman_y():
    """configs[1] graph and the reference's Y = B @ R (metrics.py:260-275)."""
    g = load_golden("roman_full")
    n = int(g["num_nodes"])
    ip, ix, d = g["indptr"], g["indices"], g["data"]
    Y, m, k = O.approx_er_projection(ip, ix, n)
    L = O.laplacian_reg(ip, ix, d, n)
    return g, n, Y, L, k


@pytest.mark.parametrize("threads", ["default", 16, 64])
def test_roman_size_column_blocks_high_threads(gs, roman_y, threads):
    """n = 22,662 with 500 CG iterations: JL columns [0, 16) and [k-16, k) solved
    on the device (the register-resident solver at T <= 16 -- 16 columns leave
    the split form 16 parts per column -- the resident one above) equal the
    oracle's CG on the same Y columns, bit for bit."""
    from gsparse.engine import blas_threads_default

    g, n, Y, L, k = roman_y
    t = blas_threads_default() if threads == "default" else threads
    data = gs.Data(edge_index=torch.from_numpy(g["edge_index"]), num_nodes=n)
    e = gs.GraphSparsifier(data, "cpu")._engine
    e.er_prepare(k)
    e.er_project_device(np.random.default_rng(42), k)
    for c0, c1 in ((0, 16), (k - 16, k)):
        Z, _ = O.cg(L, np.ascontiguousarray(Y[:, c0:c1]), 500, 1e-6, t)
        ref = O.er_from_z(g["indptr"], g["indices"], Z)
        e.er_solve(c0, c1, 500, 1e-6, t)
        got = e.er_scores(c0, c1, finalize=True)
        assert bits_equal(got, ref), (t, c0)
