"""configs[3] at full size: R-MAT-22 Jaccard-T ("Next round" item 1).

The bench's own graph (``graphs.rmat(22, 8, seed=0)``: n = 4,194,304, E =
65,245,460 directed CSR entries) through the bench's own path (device
COO -> CSR, the owner-side Jaccard of gs_jaccard.hip, the radix-select top-k):

* the device CSR equals the oracle's canonical CSR (core.py:63-76);
* device Jaccard scores bit-exact vs ``oracle_jaccard_rows`` (oracle.c: per-edge
  sorted-list merge, one fp64 divide -- metrics.py:43-62) on every entry of a
  row sample: the 64 highest-degree rows (the bitmap rows above 16,384 entries
  and the 32K-slot table class), 256 seeded random rows, and the last 64 rows of
  the CSR, whose lists end the index array (the unconditional 64-lane list steps
  read into its padding);
* the keep-0.5 device mask (core.py:229-240, device tie rule) equal to a host
  ``np.argsort(kind='stable')`` of the device's scores, and its beyond-cut /
  tie counts equal to the host's;
* the per-rank count shares of N = 2 and 8 (gs_jaccard_part_counts), scattered
  by gs_jaccard_from_counts, equal to the whole call bit for bit.
"""

from concurrent.futures import ThreadPoolExecutor
import ctypes
import os

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _host_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else (os.cpu_count() or 1)
    return max(1, min(16, n))


@pytest.fixture(scope="module")
def rmat22():
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.engine import Engine

    ei, n = graphs.rmat(22, 8, seed=0), 1 << 22
    ctx = Context(0)
    dev = torch.device("cuda", 0)
    ctx.set_graph_edge_index(n, torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev),
                             torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev))
    eng = Engine(ctx)
    scores = torch.empty(eng.nnz, dtype=torch.float64, device=dev)
    eng.jaccard(0, eng.nnz, out=scores)
    torch.cuda.synchronize(dev)
    return ei, n, ctx, eng, scores


def test_rmat22_csr_equals_oracle(rmat22):
    ei, n, ctx, eng, _ = rmat22
    ip, ix, _ = ctx.csr()
    ipo, ixo, do = O.canonical_csr(ei, n)
    assert len(ix) == 65_245_460 == ei.shape[1]  # symmetric, duplicate- and loop-free
    assert np.array_equal(ip, ipo) and np.array_equal(ix, ixo)
    assert np.all(do == 1.0)


def test_rmat22_jaccard_sampled_rows_bit_exact(rmat22):
    ei, n, ctx, eng, scores = rmat22
    ip, ix, _ = ctx.csr()
    ip = np.ascontiguousarray(ip, dtype=np.int64)
    ix = np.ascontiguousarray(ix, dtype=np.int32)
    tp, ti = O.transpose(ip, ix, n)
    deg = np.diff(ip)
    top = np.argsort(deg, kind="stable")[-64:]
    assert deg[top].max() > 16_384 and deg[top].min() > 8_192  # bitmap rows and the 32K class
    rng = np.random.default_rng(22)
    rest = rng.choice(np.setdiff1d(np.arange(n - 64), top), 256, replace=False)
    last = np.arange(n - 64, n)
    rows = np.unique(np.concatenate([top, rest, last]))
    # the last rows' lists end the index array: the device's list steps run past them
    assert ip[n] == len(ix) and deg[last].sum() > 0
    ref = np.zeros(len(ix), dtype=np.float64)
    lib = O.lib()

    def run(u):  # one row per call; rows never share a CSR entry
        lib.oracle_jaccard_rows(O._p(ip, O._i64p), O._p(ix, O._i32p), O._p(tp, O._i64p),
                                O._p(ti, O._i32p), ctypes.c_int64(int(u)), ctypes.c_int64(int(u) + 1),
                                O._p(ref, O._f64p))

    # the hubs first, so the longest merges do not finish last
    order = rows[np.argsort(-deg[rows], kind="stable")]
    with ThreadPoolExecutor(_host_threads()) as ex:
        list(ex.map(run, order.tolist()))
    sel = np.concatenate([np.arange(ip[u], ip[u + 1]) for u in rows])
    got = scores.cpu().numpy()
    assert sel.size > 1_500_000  # the hubs' entries are all in
    bad = np.flatnonzero(got[sel].view(np.uint64) != ref[sel].view(np.uint64))
    assert bad.size == 0, (bad.size, sel[bad[:8]])
    assert np.all(got[sel] >= 0.0) and np.all(got[sel] <= 1.0)


def test_rmat22_topk_keep_half_equals_stable_argsort(rmat22):
    """Jaccard-T (core.py:229-240) as the bench times it: the device radix select's
    mask == np.argsort(kind='stable') of the same scores, top int(E * 0.5)."""
    ei, n, ctx, eng, scores = rmat22
    E = ei.shape[1]
    keep = int(E * 0.5)
    mask = torch.empty(E, dtype=torch.uint8, device=scores.device)
    _, cut, beyond, tied = eng.topk_mask(scores, E, keep, False, out=mask)
    s = scores.cpu().numpy()
    ref = O.topk_mask(s, E, 0.5, False, kind="stable")
    got = mask.cpu().numpy().astype(bool)
    assert int(got.sum()) == keep
    assert np.array_equal(got, ref), int((got != ref).sum())
    assert float(cut) == float(s[ref].min())
    assert beyond == int((s > cut).sum()) and tied == int((s == cut).sum())
    assert beyond < keep <= beyond + tied  # an ambiguous cut: the tie rule decides


@pytest.mark.parametrize("nparts", [2, 8])
def test_rmat22_count_shares_rebuild_the_whole(rmat22, nparts):
    """The N-rank Jaccard (sharded_jaccard): every part's owner-pair counts, put
    together and scattered, are the one-GPU scores bit for bit."""
    ei, n, ctx, eng, scores = rmat22
    _, oo = eng.jaccard_shares(nparts)
    sizes = np.diff(oo)
    assert sizes.sum() == len(ei[0]) // 2  # each undirected pair once
    stride = int(sizes.max())
    allc = torch.zeros(nparts * stride, dtype=torch.int32, device=scores.device)
    for p in range(nparts):
        eng.jaccard_part_counts(p, nparts, out=allc[p * stride: p * stride + max(int(sizes[p]), 1)])
    out = torch.empty_like(scores)
    eng.jaccard_from_counts(nparts, allc, stride, out=out)
    assert bits_equal(out.cpu().numpy(), scores.cpu().numpy())
