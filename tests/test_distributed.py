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

    def er_prepare(self, k):
        self.k = k
        rows = O.csr_rows(self.ip)
        self.m = int(np.count_nonzero(rows < self.ix))
        return self.m

    def er_project_device(self, rng, k):
        self.Y, _, _ = O.approx_er_projection(self.ip, self.ix, self.n)

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
        bb = None
        if "backbone_jaccard" in g:
            from gsparse.distributed import sharded_backbone

            def oracle_part(ei, n, w, eps, part=0, nparts=1):
                full = O.metric_backbone(ei, n, w, eps)
                return full & ((ei[0] % nparts) == part)

            bb = sharded_backbone(comm, g["edge_index"], int(g["num_nodes"]), g["cost_jaccard"],
                                  mask_fn=oracle_part)
        if rank == 0:
            q.put((jac, jac_w, er, bb))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("name", ["karate_csr", "rmat10"])
def test_sharded_equals_single(name, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in procs:
        p.start()
    jac, jac_w, er, bb = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = load_golden(name)
    assert np.array_equal(jac.view(np.uint64), g["scores_jaccard"].view(np.uint64))
    assert np.array_equal(jac_w.view(np.uint64), g["scores_jaccard"].view(np.uint64))
    assert np.array_equal(er.view(np.uint64), g["scores_approx_er"].view(np.uint64))
    if bb is not None:
        assert np.array_equal(bb, g["backbone_jaccard"])


def test_tree_helpers():
    from gsparse.distributed import edge_ranges, pow2_floor, tree_sum

    assert edge_ranges(10, 3) == [0, 3, 6, 10]
    assert pow2_floor(6) == 4 and pow2_floor(8) == 8 and pow2_floor(1) == 1
    assert tree_sum([1.0, 2.0, 3.0, 4.0]) == (1.0 + 2.0) + (3.0 + 4.0)
