"""N>1 path on the CPU: world_size-2 (and 4) gloo process groups run the same
sharding code the MI355X bench runs over RCCL, with the oracle standing in for
each rank's device compute.  Results must equal the single-process answer
bit for bit (edge-range concat; pairwise-tree column blocks)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import gsparse_oracle as O
from conftest import load_golden


class OracleEngine:
    """Engine-shaped stand-in: the per-rank compute via the CPU oracle."""

    def __init__(self, ip, ix, d, n):
        self.ip, self.ix, self.d, self.n = ip, ix, d, n
        self.nnz = len(ix)
        self._jac = None
        rows = O.csr_rows(ip)
        fwd = np.sort(rows * n + ix)
        self.symmetric = bool(np.array_equal(fwd, np.sort(ix.astype(np.int64) * n + rows)))

    def jaccard_shares(self, nparts):
        return O.jaccard_shares(self.ip, self.ix, nparts)

    def jaccard_part_counts(self, part, nparts, out=None):
        return O.jaccard_part_counts(self.ip, self.ix, part, nparts)

    def jaccard_from_counts(self, nparts, counts, stride, out=None):
        return O.jaccard_from_counts(self.ip, self.ix, nparts, counts, stride)

    def jaccard(self, e0=0, e1=None, out=None):
        if self._jac is None:
            self._jac = O.jaccard(self.ip, self.ix)
        return self._jac[e0:e1]

    def jaccard_part(self, part, nparts, out=None):
        full = self.jaccard()
        keep = (np.arange(self.nnz) % nparts) == part
        return np.where(keep, full, 0.0)

    def degree(self, e0=0, e1=None, out=None):
        return O.degree(self.ip, self.ix, self.d)[e0:e1]

    def adamic_adar(self, e0=0, e1=None, out=None):
        return O.adamic_adar(self.ip, self.ix)[e0:e1]

    def topk_mask(self, scores, num_edges, num_keep, keep_lowest, out=None):
        """gs_topk_mask's contract: the stable-argsort mask + (cut, #beyond, #tied)."""
        s = np.asarray(scores, dtype=np.float64)
        mask = np.zeros(num_edges, dtype=bool)
        if num_keep <= 0:
            if not keep_lowest:
                mask[: len(s)] = True
            return mask, float("nan"), (0 if keep_lowest else len(s)), 0
        idx = np.argsort(s, kind="stable")
        sel = idx[:num_keep] if keep_lowest else idx[-num_keep:]
        mask[sel] = True
        cut = s[sel[-1]] if keep_lowest else s[sel[0]]
        beyond = int((s < cut).sum()) if keep_lowest else int((s > cut).sum())
        return mask, float(cut), beyond, int((s == cut).sum())

    # gs_jsel_*'s contract (include/gsparse.h), restated with NumPy: keys of this part's
    # owner pairs, weighted radix histograms (12 + 4 x 13 bits), keep bytes, the mask
    JSEL_BINS, JSEL_PASSES = 8192, 5

    def _owners(self):
        ip, ix = np.asarray(self.ip, dtype=np.int64), np.asarray(self.ix, dtype=np.int64)
        rows = O.csr_rows(ip)
        deg = np.diff(ip)
        own = (deg[rows] > deg[ix]) | ((deg[rows] == deg[ix]) & (rows <= ix))
        e = np.nonzero(own)[0]
        rev = np.searchsorted(rows * self.n + ix, ix[e] * self.n + rows[e])
        return e, rev, deg[rows[e]] + deg[ix[e]]

    @staticmethod
    def _key(v):
        b = np.asarray(v, dtype=np.float64).view(np.uint64)
        return np.where(b >> np.uint64(63), ~b, b | np.uint64(1 << 63))

    def _hist(self, p):
        shift, bits = (52, 12) if p == 0 else (52 - 13 * p, 13)
        top = shift + bits
        hmask = np.uint64(0) if top >= 64 else np.uint64(((1 << 64) - 1) ^ ((1 << top) - 1))
        sel = (self._keys & hmask) == (np.uint64(self._prefix) & hmask)
        d = (self._keys[sel] >> np.uint64(shift)) & np.uint64((1 << bits) - 1)
        return np.bincount(d.astype(np.int64), weights=self._wt[sel], minlength=self.JSEL_BINS).astype(np.int64)

    def jsel_begin(self, part, nparts, counts, num_keep, keep_lowest, hist, scores=None):
        _, Oo = self.jaccard_shares(nparts)
        a, b = int(Oo[part]), int(Oo[part + 1])
        opos, orev, osum = (x[a:b] for x in self._owners())
        cnt = np.asarray(counts[: b - a].numpy() if hasattr(counts, "numpy") else counts[: b - a],
                         dtype=np.int64).astype(np.uint32).astype(np.float64)
        uni = osum.astype(np.float64) - cnt
        val = np.divide(cnt, uni, out=np.zeros_like(cnt), where=uni > 0)
        self._keys, self._wt, self._pp = self._key(val), np.where(opos == orev, 1, 2), (opos, orev)
        self._lowest, self._prefix, self._below, self._eq, self._pass = keep_lowest, 0, 0, 0, 0
        self._rank = num_keep - 1 if keep_lowest else self.nnz - num_keep
        hist.copy_(torch.from_numpy(self._hist(0)))
        if scores is not None:
            scores[: b - a] = torch.from_numpy(val)
        return b - a

    def jsel_step(self, hist):
        p = self._pass
        h = hist.numpy().astype(np.int64)[: 1 << (12 if p == 0 else 13)]
        c = np.cumsum(h)
        d = int(np.searchsorted(c, self._rank, side="right"))
        acc = int(c[d - 1]) if d else 0
        self._rank -= acc
        self._below += acc
        self._prefix |= d << (52 if p == 0 else 52 - 13 * p)
        self._pass += 1
        if self._pass == self.JSEL_PASSES:
            self._eq = int(h[d])
        else:
            hist.copy_(torch.from_numpy(self._hist(self._pass)))
        return self.JSEL_PASSES - self._pass

    def jsel_result(self):
        cut = int(self._prefix)
        b = cut & ((1 << 63) - 1) if cut >> 63 else ~cut & ((1 << 64) - 1)
        nb = self._below if self._lowest else self.nnz - self._below - self._eq
        tied = self._keys == np.uint64(cut)
        opos, orev = self._pp
        self._tpos = np.concatenate([opos[tied], orev[tied & (orev != opos)]])
        return float(np.array([b], dtype=np.uint64).view(np.float64)[0]), nb, self._eq, len(self._tpos)

    def jsel_tie_positions(self, out):
        out[: len(self._tpos)] = torch.from_numpy(self._tpos)
        return out

    def jsel_keep(self, tie_pos, ntie, need, out):
        cut = np.uint64(self._prefix)
        k = self._keys
        opos, orev = self._pp
        beyond = (k < cut) if self._lowest else (k > cut)
        b = np.where(beyond, 3, 0).astype(np.uint8)
        tied = k == cut
        if need >= ntie:
            b[tied] = 3
        elif need > 0:
            t = np.sort(tie_pos.numpy())
            ra, rb = np.searchsorted(t, opos[tied]), np.searchsorted(t, orev[tied])
            ka = ra < need if self._lowest else ra >= ntie - need
            kb = rb < need if self._lowest else rb >= ntie - need
            b[tied] = ka.astype(np.uint8) | (kb.astype(np.uint8) << 1)
        b4 = np.zeros((len(b) + 3) // 4 * 4, dtype=np.uint8)  # four 2-bit codes per byte
        b4[: len(b)] = b
        b4 = b4.reshape(-1, 4)
        packed = (b4[:, 0] | (b4[:, 1] << 2) | (b4[:, 2] << 4) | (b4[:, 3] << 6)).astype(np.uint8)
        out[: len(packed)] = torch.from_numpy(packed)
        return out

    def jsel_mask(self, nparts, keep_all, stride, out):
        _, Oo = self.jaccard_shares(nparts)
        opos, orev, _ = self._owners()
        i = np.arange(len(opos))
        r = np.searchsorted(Oo, i, side="right") - 1
        c = 4 * r * stride + (i - Oo[r])
        kb = (keep_all.numpy()[c >> 2] >> (2 * (c & 3))) & 3
        m = np.zeros(self.nnz, dtype=np.uint8)
        m[orev] = (kb >> 1) & 1
        m[opos] = np.where(orev == opos, kb & 1, kb & 1)
        out[: self.nnz] = torch.from_numpy(m)
        return out

    def er_prepare(self, k):
        self.k = k
        rows = O.csr_rows(self.ip)
        self.m = int(np.count_nonzero(rows < self.ix))
        return self.m

    def er_project_device(self, rng, k, cols=None):
        Y, _, _ = O.approx_er_projection(self.ip, self.ix, self.n)
        c0, c1 = cols if cols is not None else (0, k)
        self.Y = np.full_like(Y, np.nan)  # columns outside the slice must not be read
        self.Y[:, c0:c1] = Y[:, c0:c1]

    er_project_host = er_project_device

    def er_solve(self, c0, c1, maxiter, tol, threads):
        L = O.laplacian_reg(self.ip, self.ix, self.d, self.n)
        self.c0 = c0
        self.Z, _ = O.cg(L, np.ascontiguousarray(self.Y[:, c0:c1]), maxiter, tol, threads)

    def er_scores(self, c0, c1, finalize=False, out=None):
        rows = O.csr_rows(self.ip)
        Z = self.Z[:, c0 - self.c0:c1 - self.c0]
        diff = Z[rows] - Z[self.ix]
        return np.sum(diff ** 2, axis=1)


class OracleStages:
    """gs_bb_*'s protocol (metric_backbone.BackboneStages) with the CPU oracle as each
    rank's compute: the landmark labels of this rank's landmarks (l = rank mod N) must
    come back whole from the MIN / MAX exchange, certify decides every third column of
    the rank's column range, and search decides the columns of the sources of this
    rank's batches (every N-th of each range, the batches taken from the last as the
    library's ascending-count order takes them).  What is tested is the exchange: the
    stages' ranges and the all-reduces must leave every column decided, and the mask
    equal to the reference's."""

    def __init__(self, S=2):
        self.S = S

    def begin(self, ei, n, w, eps, part, nparts):
        self.ei = np.asarray(ei, dtype=np.int64)
        self.n, self.E = n, self.ei.shape[1]
        self.full = O.metric_backbone(self.ei, n, w, eps)
        self.state = np.zeros(self.E, dtype=np.uint8)
        self.K = 3
        self.D = np.full(self.K * n, np.inf)
        self.comp = np.zeros(self.K, dtype=np.int32)
        for l in range(part, self.K, nparts):
            self.D[l::self.K] = float(l)
            self.comp[l] = 1
        return self.K

    def landmarks_io(self, D, comp, out):
        if out:
            D.copy_(torch.from_numpy(self.D))
            comp.copy_(torch.from_numpy(self.comp))
        else:
            self.D, self.comp = D.numpy().copy(), comp.numpy().copy()

    def certify(self, part, nparts):
        assert np.array_equal(self.D, np.tile(np.arange(self.K, dtype=np.float64), self.n))
        assert (self.comp == 1).all()
        c0, c1 = self.E * part // nparts, self.E * (part + 1) // nparts
        idx = np.arange(c0, c1)
        idx = idx[idx % 3 == 0]
        self.state[idx] = np.where(self.full[idx], 1, 2)

    def state_io(self, st, out):
        if out:
            st.copy_(torch.from_numpy(self.state))
        else:
            self.state = st.numpy().copy()

    def plan(self):
        self.sources = np.unique(self.ei[0][self.state == 0])
        self.nbatch = (len(self.sources) + self.S - 1) // self.S
        return self.nbatch

    def search(self, b0, b1, part, nparts):
        for bq in range(b0 + part, b1, nparts):
            bi = self.nbatch - 1 - bq
            for u in self.sources[bi * self.S:(bi + 1) * self.S]:
                cols = (self.ei[0] == u) & (self.state == 0)
                self.state[cols] = np.where(self.full[cols], 1, 2)

    def finish(self, keep):
        assert (self.state != 0).all(), int((self.state == 0).sum())
        keep[: self.E] = torch.from_numpy((self.state == 1).astype(np.uint8))
        return keep, 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gsparse.distributed import Comm, sharded_approx_er, sharded_edge_scores, work_ranges

        g = load_golden(name)
        eng = OracleEngine(g["indptr"], g["indices"], g["data"], int(g["num_nodes"]))
        comm = Comm()
        jac = sharded_edge_scores(eng, comm, "jaccard").numpy()
        jac_w = sharded_edge_scores(eng, comm, "jaccard",
                                    bounds=work_ranges(g["indptr"], g["indices"], world)).numpy()
        er = sharded_approx_er(eng, comm, blas_threads=1).numpy()
        from gsparse.distributed import sharded_sparsify

        E = g["edge_index"].shape[1]
        masks = {}
        for r in (0.8, 0.5, 0.2):
            for low in (False, True):
                for tb in ("numpy", "stable"):
                    m, _ = sharded_sparsify(eng, comm, torch.from_numpy(jac), E, r, low, tie_break=tb)
                    masks[(r, low, tb)] = m.numpy().copy()
        # Jaccard-T without the score exchange (gs_jsel_* protocol): the same kept sets
        from gsparse.distributed import sharded_jaccard_topk

        nnz = len(g["indices"])
        jsel = {}
        for r in (0.8, 0.5, 0.2):
            for low in (False, True):
                for tb in ("numpy", "stable"):
                    m, info, sc = sharded_jaccard_topk(eng, comm, r, low, tie_break=tb)
                    jsel[(r, low, tb)] = m[:nnz].numpy().astype(bool)
                    if E == nnz:
                        assert np.array_equal(jsel[(r, low, tb)], masks[(r, low, tb)]), (r, low, tb, info)
        bb = None
        if "backbone_jaccard" in g:
            from gsparse.distributed import sharded_backbone

            bb = sharded_backbone(comm, g["edge_index"], int(g["num_nodes"]), g["cost_jaccard"],
                                  stages=OracleStages())
            # one range per batch: an exchange after every batch of N ranks
            bb1 = sharded_backbone(comm, g["edge_index"], int(g["num_nodes"]), g["cost_jaccard"],
                                   stages=OracleStages(S=1), phases=[i / 7 for i in range(1, 7)])
            assert np.array_equal(bb, bb1)
            # ranks asking for different search ranges follow rank 0's (no
            # mismatched collective counts)
            bb2 = sharded_backbone(comm, g["edge_index"], int(g["num_nodes"]), g["cost_jaccard"],
                                   stages=OracleStages(), phases=[0.3] if rank == 0 else [0.5, 0.7])
            assert np.array_equal(bb, bb2)
        # every rank selected the same kept set
        allm = [None] * world
        dist.all_gather_object(allm, {k: v.tobytes() for k, v in masks.items()})
        assert all(a == allm[0] for a in allm)
        if rank == 0:
            q.put((jac, jac_w, er, bb, masks, jsel))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("name", ["karate_csr", "rmat10", "roman2000"])
def test_sharded_equals_single(name, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    jac, jac_w, er, bb, masks, jsel = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = load_golden(name)
    assert np.array_equal(jac.view(np.uint64), g["scores_jaccard"].view(np.uint64))
    assert np.array_equal(jac_w.view(np.uint64), g["scores_jaccard"].view(np.uint64))
    assert np.array_equal(er.view(np.uint64), g["scores_approx_er"].view(np.uint64))
    if bb is not None:
        assert np.array_equal(bb, g["backbone_jaccard"])
    # the global top-k after the all-gather: the reference's masks (numpy ties) and
    # np.argsort(kind='stable') (device tie rule), core.py:229-240
    E = g["edge_index"].shape[1]
    for (r, low, tb), m in masks.items():
        if tb == "numpy" and f"mask_jaccard_{r}_{int(low)}" in g:
            assert np.array_equal(m, g[f"mask_jaccard_{r}_{int(low)}"]), (r, low)
        if tb == "stable":
            assert np.array_equal(m, O.topk_mask(g["scores_jaccard"], E, r, low, kind="stable")), (r, low)
    # the distributed select over CSR entries: np.argsort(kind='stable') of the scores
    nnz = len(g["indices"])
    for (r, low, tb), m in jsel.items():
        if tb == "stable":
            assert np.array_equal(m, O.topk_mask(g["scores_jaccard"], nnz, r, low, kind="stable")), (r, low)


def test_tree_helpers():
    from gsparse.distributed import dyadic_cover, edge_ranges, pow2_floor, tree_sum

    assert edge_ranges(10, 3) == [0, 3, 6, 10]
    assert pow2_floor(6) == 4 and pow2_floor(8) == 8 and pow2_floor(1) == 1
    assert tree_sum([1.0, 2.0, 3.0, 4.0]) == (1.0 + 2.0) + (3.0 + 4.0)
    from gsparse.distributed import fold_pairwise

    rng = np.random.default_rng(3)
    for cnt in (1, 2, 4, 8, 16):
        parts = [rng.standard_normal(5) * 10.0 ** rng.integers(-8, 8) for _ in range(cnt)]
        assert np.array_equal(fold_pairwise(iter(parts)), tree_sum(parts))
    with pytest.raises(ValueError):
        fold_pairwise([1.0, 2.0, 3.0])
    assert dyadic_cover(0, 32) == [(5, 0)]
    assert dyadic_cover(5, 11) == [(0, 5), (1, 3), (1, 4), (0, 10)]
    assert dyadic_cover(3, 3) == []


@pytest.mark.parametrize("world", [1, 2, 3, 5, 6, 7, 8])
def test_er_rank_blocks_cover_k(world):
    """Every rank's columns are whole pairwise-tree nodes and together cover k once."""
    from gsparse.distributed import dyadic_cover, er_rank_blocks

    for k in (2674, 3210, 2107, 4066, 300, 100):
        d, b, runs = er_rank_blocks(k, world)
        assert len(b) == (1 << d) + 1 and b[0] == 0 and b[-1] == k
        assert runs[0][0] == 0 and runs[-1][1] == len(b) - 1
        assert all(runs[r][1] == runs[r + 1][0] for r in range(world - 1))
        for a, z in runs:
            cov = dyadic_cover(a, z)
            assert sum(1 << lev for lev, _ in cov) == z - a


@pytest.mark.parametrize("nparts", [1, 2, 3, 8])
@pytest.mark.parametrize("name", ["karate_csr", "rmat10", "roman2000", "star", "triangle"])
def test_jaccard_count_shares_rebuild_scores(name, nparts):
    """Owner-pair counts of every part, scattered, are the reference's Jaccard bit for bit."""
    g = load_golden(name)
    ip, ix = g["indptr"], g["indices"]
    R, Oo = O.jaccard_shares(ip, ix, nparts)
    assert R[0] == 0 and R[-1] == len(ip) - 1 and np.all(np.diff(R) >= 0)
    parts = [O.jaccard_part_counts(ip, ix, p, nparts) for p in range(nparts)]
    assert [len(p) for p in parts] == list(np.diff(Oo))
    stride = max(1, max(len(p) for p in parts))
    allc = np.zeros(nparts * stride, dtype=np.uint32)
    for p, c in enumerate(parts):
        allc[p * stride: p * stride + len(c)] = c
    got = O.jaccard_from_counts(ip, ix, nparts, allc, stride)
    assert np.array_equal(got.view(np.uint64), g["scores_jaccard"].view(np.uint64))
