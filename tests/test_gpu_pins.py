"""GPU pins of exactly what bench.py times ("Next round" item 1).

* ApproxER at configs[1] size in the bench's own configuration: the Roman-like
  graph, k = 2,674 JL columns, 500 CG iterations, the OpenBLAS ddot order of 8
  threads (``--blas-threads`` default) and of 16 (the box's default, the drop-in
  API's order), the default CG mode (5: the
  register-resident solver).  The whole solve runs as the bench runs it, then
  the first round of whole columns (``k_cg_regwide<2,44>``, columns [0, 256))
  and the last, partly occupied round (columns [2560, 2674): whole columns inside the
  same launch since round 6; the split form is pinned by the forced-split parity
  tests) are read back and compared bit for bit with the oracle's CG (oracle.c: SciPy 1.15's
  recurrence, OpenBLAS-SkylakeX ddot for 8 threads) on the same Y columns.
  Reference: metrics.py:272-289.
* The metric backbone (configs[4]) at the bench's sizes: the full Roman-like
  graph against the oracle's bounded Dijkstra over every row, and R-MAT-18 on
  sampled source rows (the 8 highest-degree rows + 56 seeded random rows):
  every column of those rows against a per-row Dijkstra cut at the row's
  largest target cost.  Reference: metric_backbone.py:86, 97-111.
"""

from concurrent.futures import ThreadPoolExecutor
import os

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal

pytestmark = pytest.mark.gpu


def _host_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else (os.cpu_count() or 1)
    return max(1, min(16, n))


@pytest.fixture(scope="module", params=[8, 16])
def roman_t8(request):
    """The bench's Roman step (bench.py main(): er_prepare -> device normal stream ->
    er_solve(0, k, 500, 1e-6, T)), with Z of the two pinned column blocks: T = 8 (the
    headline's OpenBLAS order) and T = 16 (the box's default thread count, the drop-in
    API's order -- bench.py's box_blas_order line)."""
    T = request.param
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.engine import Engine, jl_dim

    ei, n = graphs.roman_like(), 22_662
    ctx = Context(0)
    ctx.set_graph_edge_index(n, np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1]))
    eng = Engine(ctx)
    k = jl_dim(n, 0.3)
    assert k == 2674
    ctx.profile(True)
    ctx.profile_reset()
    eng.er_prepare(k)
    eng.er_project_device(np.random.default_rng(42), k)
    eng.er_solve(0, k, 500, 1e-6, T)
    prof = ctx.profile_read()
    ctx.profile(False)
    blocks = {"first_round": (0, 256), "split_tail": (2560, k)}
    z = {name: eng.er_z(a, b) for name, (a, b) in blocks.items()}
    its = eng.er_iterations()
    scores = eng.er_scores(0, k, True)
    return ei, n, k, blocks, z, its, prof, scores, T


@pytest.fixture(scope="module")
def roman_oracle_y():
    from gsparse import graphs

    ei, n = graphs.roman_like(), 22_662
    ip, ix, d = O.canonical_csr(ei, n)
    Y, m, k = O.approx_er_projection(ip, ix, n)
    return ip, ix, d, Y, O.laplacian_reg(ip, ix, d, n)


def _oracle_cg_columns(L, Y, cols, blas_threads=8):
    """O.cg on the listed columns, spread over host threads (ctypes drops the GIL)."""
    th = _host_threads()
    groups = [cols[i::th] for i in range(th) if len(cols[i::th])]

    def run(c):
        return c, O.cg(L, Y[:, c], 500, 1e-6, blas_threads)

    Z = np.empty((Y.shape[0], len(cols)), dtype=np.float64)
    its = np.empty(len(cols), dtype=np.int32)
    pos = {c: i for i, c in enumerate(cols)}
    with ThreadPoolExecutor(len(groups)) as ex:
        for c, (z, it) in ex.map(run, groups):
            idx = [pos[x] for x in c]
            Z[:, idx] = z
            its[idx] = it
    return Z, its


def test_roman_t8_solve_takes_the_timed_kernels(roman_t8):
    """The solve ran the register-resident launch (cg_reg) and the split tail did
    not fall back (no hand-off abort): the kernels pinned below are the bench's."""
    *_, prof, _, _ = roman_t8
    assert "cg_reg" in prof, prof
    assert "cg_split_abort" not in prof, prof


@pytest.mark.parametrize("block", ["first_round", "split_tail"])
def test_roman_t8_columns_bit_exact_vs_oracle_cg(roman_t8, roman_oracle_y, block):
    """Z columns of the timed T = 8 solve == the oracle's CG, bit for bit
    (metrics.py:284-289; north_star float tolerance 1e-5 asserted beside it)."""
    _, n, k, blocks, z, its, _, _, T = roman_t8
    _, _, _, Y, L = roman_oracle_y
    a, b = blocks[block]
    cols = list(range(a, b))
    Zo, ito = _oracle_cg_columns(L, Y, cols, blas_threads=T)
    assert np.array_equal(its[a:b], ito)
    assert (ito == 500).all()  # chain-like graph: every column runs to maxiter
    got = z[block]
    rel = float(np.max(np.abs(got - Zo) / np.maximum(np.abs(Zo), 1e-300)))
    assert rel <= 1e-5, rel
    bad = np.nonzero(got.view(np.uint64) != Zo.view(np.uint64))
    assert bits_equal(got, Zo), (len(bad[0]), rel)


def test_roman_t8_scores_from_pinned_blocks(roman_t8, roman_oracle_y):
    """Sanity of the read-out path: scores of the timed solve are finite, positive
    and clamped as metrics.py:293-297 clamps."""
    *_, scores, _ = roman_t8
    assert np.isfinite(scores).all() and (scores >= 1e-10).all()


def _bench_costs(ei, n, scores=None):
    """bench_backbone's costs: _scores_to_cost(Jaccard) in CSR order, [:E]."""
    ip, ix, _ = O.canonical_csr(ei, n)
    s = O.jaccard(ip, ix) if scores is None else scores
    return O.scores_to_cost(s, "jaccard")[: ei.shape[1]], ip, ix


def test_backbone_roman_full_vs_oracle():
    """configs[4], Roman-like: the device keep mask == the oracle's bounded
    Dijkstra over every source row, for Jaccard, Adamic-Adar and degree costs."""
    import gsparse
    from gsparse import graphs
    from gsparse.metric_backbone import backbone_mask

    ei, n = graphs.roman_like(), 22_662
    E = ei.shape[1]
    w, ip, ix = _bench_costs(ei, n)
    keep = backbone_mask(ei, n, w)
    ref = O.metric_backbone(ei, n, w)
    assert np.array_equal(keep, ref)
    assert 0 < ref.sum() < E
    data = gsparse.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    _, st = gsparse.compute_metric_backbone(data, w, epsilon=1e-9, verbose=False)
    assert np.array_equal(st["keep_mask"], ref)
    d = O.canonical_csr(ei, n)[2]
    for metric, s in (("adamic_adar", O.adamic_adar(ip, ix)), ("degree", O.degree(ip, ix, d))):
        wm = O.scores_to_cost(s, metric)[:E]
        assert np.array_equal(backbone_mask(ei, n, wm), O.metric_backbone(ei, n, wm)), metric


def test_backbone_rmat18_sampled_rows_vs_oracle():
    """configs[4], R-MAT-18 (the bench's graph, E = 3,938,716): every column of 64
    source rows (the 8 highest-degree rows + 56 seeded random rows) against a
    bounded Dijkstra per row (oracle.c) cut at the row's largest target cost."""
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.engine import Engine
    from gsparse.metric_backbone import backbone_mask

    ei, n = graphs.rmat(18, 8, seed=0), 1 << 18
    ctx = Context(0)
    ctx.set_graph_edge_index(n, np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1]))
    jac = Engine(ctx).jaccard()  # bit-exact vs the oracle (test_gpu_parity); oracle.c takes ~25 s here
    w, ip, _ = _bench_costs(ei, n, scores=jac)
    keep = backbone_mask(ei, n, w)
    deg = np.diff(ip)
    top = np.argsort(deg, kind="stable")[-8:]
    rest = np.random.default_rng(18).choice(np.setdiff1d(np.arange(n), top), 56, replace=False)
    src = np.concatenate([top, rest])
    ref, decided = O.metric_backbone_rows(ei, n, w, src, threads=_host_threads())
    assert decided.sum() >= deg[top].sum()  # the hubs' columns are all in
    assert np.array_equal(keep[decided], ref[decided]), int((keep[decided] != ref[decided]).sum())
    assert 0 < ref[decided].sum() < decided.sum()
