"""Multi-GPU sharding of the scorers (one process per GPU, torch.distributed).

SURVEY §8(e):
  * Jaccard on a symmetric graph: each rank takes its share of the owner-side
    pair tasks (gs_jaccard_part: both CSR entries of a pair, zeros elsewhere)
    and one all-reduce(sum) assembles the whole vector -- exact, since every
    entry has exactly one non-zero contributor.
  * metric backbone: the per-source searches by source row (u % world), one
    all-reduce(sum) of the keep bytes.
  * AA / degree / FeatCos (and Jaccard on explicit ranges): contiguous CSR
    edge ranges (equal counts, or equal per-edge work d_u + d_v for skewed
    graphs), then an all-gather of the fp64 scores so every rank can run the
    global top-k.
  * ApproxER: the k JL columns are independent CG solves.  Rank blocks are
    nodes of NumPy's pairwise-sum tree over k (gs_er_split), so each rank's
    per-edge partial sum is exactly a subtree of the reference's
    ``np.sum(diff**2, axis=1)``; partials are all-gathered and added in tree
    order -- scores are bit-identical for any power-of-two rank count.
The RCCL backend ("nccl") moves device tensors over xGMI; "gloo" (CPU
tensors) runs the same code for tests and rehearsals.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def edge_ranges(nnz: int, world: int) -> list[int]:
    """Equal-count contiguous CSR edge ranges."""
    return [nnz * r // world for r in range(world + 1)]


def work_ranges(indptr: np.ndarray, indices: np.ndarray, world: int) -> list[int]:
    """Contiguous edge ranges cut at equal prefix sums of d_u + d_v."""
    deg = np.diff(indptr)
    rows = np.repeat(np.arange(len(deg)), deg)
    w = (deg[rows] + deg[indices]).astype(np.float64)
    cw = np.cumsum(w)
    total = cw[-1] if len(cw) else 0.0
    b = [0]
    for r in range(1, world):
        b.append(int(np.searchsorted(cw, total * r / world)))
    b.append(len(indices))
    return b


def pow2_floor(x: int) -> int:
    p = 1
    while p * 2 <= x:
        p *= 2
    return p


def tree_sum(parts):
    """Combine per-block partial sums in NumPy pairwise-tree order."""
    parts = list(parts)
    while len(parts) > 1:
        parts = [parts[i] + parts[i + 1] for i in range(0, len(parts), 2)]
    return parts[0]


def finalize_er(total):
    """metrics.py:293-297 on the tree-combined sum (0 + s, nan_to_num, clamp)."""
    t = 0.0 + total
    if isinstance(t, torch.Tensor):
        return torch.nan_to_num(t, nan=1e-10, posinf=1e-10, neginf=1e-10).clamp_min(1e-10)
    t = np.nan_to_num(t, nan=1e-10, posinf=1e-10, neginf=1e-10)
    return np.maximum(t, 1e-10)


class Comm:
    """Thin wrapper: device tensors for nccl (RCCL), CPU tensors for gloo."""

    def __init__(self, group=None, device: torch.device | None = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.device = device if (device is not None and self.backend == "nccl") \
            else torch.device("cpu")

    def tensor(self, x) -> torch.Tensor:
        if isinstance(x, np.ndarray):
            x = torch.from_numpy(np.ascontiguousarray(x))
        return x.to(self.device)

    def all_gather_padded(self, local: torch.Tensor, sizes: list[int]) -> torch.Tensor:
        """Concatenate variable-length 1-D shards (sizes known everywhere)."""
        mx = max(sizes) if sizes else 0
        buf = torch.zeros(mx, dtype=local.dtype, device=self.device)
        buf[: local.numel()] = local.to(self.device)
        out = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(out, buf, group=self.group)
        return torch.cat([out[r][: sizes[r]] for r in range(self.world)])

    def all_reduce_sum(self, local: torch.Tensor) -> torch.Tensor:
        t = local.to(self.device).clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def all_gather_same(self, local: torch.Tensor) -> list[torch.Tensor]:
        out = [torch.empty_like(local, device=self.device) for _ in range(self.world)]
        dist.all_gather(out, local.to(self.device), group=self.group)
        return out


def sharded_edge_scores(engine, comm: Comm, metric: str, bounds: list[int] | None = None,
                        **kw):
    """One scorer over this rank's CSR edge range, all-gathered to every rank."""
    nnz = engine.nnz
    if metric == "jaccard" and bounds is None and hasattr(engine, "jaccard_part"):
        out = None
        if comm.device.type == "cuda":
            out = torch.empty(nnz, dtype=torch.float64, device=comm.device)
        part = engine.jaccard_part(comm.rank, comm.world, out=out)
        return comm.all_reduce_sum(comm.tensor(part))
    b = bounds or edge_ranges(nnz, comm.world)
    e0, e1 = b[comm.rank], b[comm.rank + 1]
    fn = {"jaccard": engine.jaccard, "adamic_adar": engine.adamic_adar,
          "degree": engine.degree}.get(metric)
    out = None
    if comm.device.type == "cuda":
        out = torch.empty(e1 - e0, dtype=torch.float64, device=comm.device)
    if metric == "feature_cosine":
        local = engine.feature_cosine(kw["x"], e0, e1, out=out)
    elif fn is not None:
        local = fn(e0, e1, out=out)
    else:
        raise ValueError(metric)
    sizes = [b[r + 1] - b[r] for r in range(comm.world)]
    return comm.all_gather_padded(comm.tensor(local), sizes)


def sharded_backbone(comm: Comm, edge_index: np.ndarray, num_nodes: int,
                     edge_weights: np.ndarray, epsilon: float = 1e-9, mask_fn=None) -> np.ndarray:
    """metric_backbone keep mask with the per-source searches split over ranks
    (source row u goes to rank u % world); one all-reduce(sum) of the keep
    bytes -- each column is decided by exactly one rank."""
    from .metric_backbone import check_weights

    check_weights(edge_weights, np.asarray(edge_index).shape[1])
    if mask_fn is None:
        from .metric_backbone import backbone_mask as mask_fn
    part = mask_fn(edge_index, num_nodes, edge_weights, epsilon, part=comm.rank,
                   nparts=comm.world)
    t = comm.tensor(np.ascontiguousarray(part, dtype=np.uint8).astype(np.int32))
    return comm.all_reduce_sum(t).cpu().numpy().astype(bool)


def sharded_approx_er(engine, comm: Comm, epsilon: float = 0.3, seed: int = 42,
                      max_cg_iters: int = 500, cg_tol: float = 1e-6, blas_threads: int = 1,
                      rng_mode: str = "device"):
    """ApproxER with the JL columns split over ranks along the pairwise tree."""
    from .engine import er_split, jl_dim

    n = engine.n
    k = jl_dim(n, epsilon)
    rng = np.random.default_rng(seed)
    m = engine.er_prepare(k)
    if m == 0:
        return comm.tensor(np.zeros(engine.nnz))
    parts = pow2_floor(comm.world)
    bounds = [0, k]
    while parts > 1:  # every block must be a non-leaf node of the pairwise tree
        try:
            bounds = er_split(k, parts)
            break
        except ValueError:
            parts //= 2
    if rng_mode == "device":
        engine.er_project_device(rng, k)
    else:
        engine.er_project_host(rng, k)
    if comm.rank < parts:
        c0, c1 = bounds[comm.rank], bounds[comm.rank + 1]
        engine.er_solve(c0, c1, max_cg_iters, cg_tol, blas_threads)
        out = None
        if comm.device.type == "cuda":
            out = torch.empty(engine.nnz, dtype=torch.float64, device=comm.device)
        local = comm.tensor(engine.er_scores(c0, c1, finalize=False, out=out))
    else:
        local = comm.tensor(np.zeros(engine.nnz))
    gathered = comm.all_gather_same(local)
    return finalize_er(tree_sum(gathered[:parts]))
