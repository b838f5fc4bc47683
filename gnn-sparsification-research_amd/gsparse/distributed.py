"""Multi-GPU sharding of the scorers (one process per GPU, torch.distributed).

SURVEY §8(e):
  * Jaccard on a symmetric graph: each undirected pair is intersected once, at
    its owner endpoint; rank r takes the owner pairs of a contiguous row range
    cut at equal shares of the intersection work (gs_jaccard_shares, the same
    on every rank) and produces their integer counts (gs_jaccard_part_counts,
    4 B per pair).  One all-gather of the counts, then every rank writes the
    score of both CSR entries of every pair (gs_jaccard_from_counts: the
    reference's single fp64 division) -- 2 B per directed edge on the wire
    instead of the 8 B per edge of a score all-gather.
  * metric backbone, in stages (gs_bb_*): the landmark searches split over the
    ranks (MIN all-reduce of their labels), the columns' witnesses and
    certificates by range, then the searches by source -- every rank's every
    N-th batch of each range of the ascending-count order -- with a MAX
    all-reduce of the column-state bytes after each stage.
  * AA / degree / FeatCos (and Jaccard on explicit ranges): contiguous CSR
    edge ranges (equal counts, or equal per-edge work d_u + d_v for skewed
    graphs), then an all-gather of the fp64 scores so every rank can run the
    global top-k.
  * the global top-k (sharded_sparsify): every rank holds the all-gathered
    scores and runs the same radix select on its own device -- the kept set is
    identical on every rank and to one GPU's, with no further exchange.
  * Jaccard-T without the score exchange (sharded_jaccard_topk): the ranks radix-select
    the cut over their own owner pairs with all-reduced histograms (gs_jsel_*), then
    all-gather one keep byte per pair -- no replicated score scatter or full top-k.
  * ApproxER: the k JL columns are independent CG solves.  Rank blocks are
    nodes of NumPy's pairwise-sum tree over k (gs_er_split), so each rank's
    per-edge partial sum is exactly a subtree of the reference's
    ``np.sum(diff**2, axis=1)``; partials are all-gathered and added in tree
    order.  A power-of-two rank count takes one tree node per rank; any other
    count takes contiguous runs of the nodes one level deeper than needed (down
    to the tree's leaves) and sends the partial sums of the maximal subtrees of
    its run, combined in tree order on every rank -- bit-identical for any N.
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


def fold_pairwise(parts):
    """tree_sum of a power-of-two number of parts, folded as they arrive: a stack of
    at most log2(count) + 1 partial sums instead of every part at once."""
    stack = []
    for p in parts:
        stack.append((1, p))
        while len(stack) >= 2 and stack[-1][0] == stack[-2][0]:
            (s, right), (_, left) = stack.pop(), stack.pop()
            stack.append((2 * s, left + right))
    if len(stack) != 1:
        raise ValueError("fold_pairwise needs a power-of-two number of parts")
    return stack[0][1]


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

    def broadcast_from(self, t: torch.Tensor, src: int) -> torch.Tensor:
        """Broadcast from group rank `src` (in place on the receivers)."""
        g = src if self.group is None else dist.get_global_rank(self.group, src)
        dist.broadcast(t, src=g, group=self.group)
        return t

    def all_gather_flat(self, local: torch.Tensor) -> torch.Tensor:
        """Equal-size shards concatenated in rank order (one RCCL all-gather
        into a flat buffer; gloo: list all-gather + cat)."""
        local = local.to(self.device).contiguous()
        if self.backend == "nccl":
            out = torch.empty(self.world * local.numel(), dtype=local.dtype, device=self.device)
            dist.all_gather_into_tensor(out, local, group=self.group)
            return out
        return torch.cat(self.all_gather_same(local))


def sharded_jaccard(engine, comm: Comm, out=None):
    """Jaccard of a symmetric graph over ranks: this rank's owner-pair counts,
    one all-gather of the uint32 counts (padded to the largest share), scores of
    every CSR entry on every rank -- bit-identical to engine.jaccard()."""
    _, oo = engine.jaccard_shares(comm.world)
    sizes = np.diff(oo)
    stride = max(1, int(sizes.max()) if len(sizes) else 1)
    if comm.device.type == "cuda":
        buf = torch.zeros(stride, dtype=torch.int32, device=comm.device)
        engine.jaccard_part_counts(comm.rank, comm.world, out=buf)
    else:
        buf = torch.zeros(stride, dtype=torch.int32)
        part = np.asarray(engine.jaccard_part_counts(comm.rank, comm.world), dtype=np.uint32)
        buf[: part.shape[0]] = torch.from_numpy(part.view(np.int32))
    allc = comm.all_gather_flat(buf)
    if comm.device.type == "cuda":
        if out is None:
            out = torch.empty(engine.nnz, dtype=torch.float64, device=comm.device)
        return engine.jaccard_from_counts(comm.world, allc, stride, out=out)
    return torch.from_numpy(np.asarray(
        engine.jaccard_from_counts(comm.world, allc.numpy().view(np.uint32), stride)))


def sharded_edge_scores(engine, comm: Comm, metric: str, bounds: list[int] | None = None,
                        **kw):
    """One scorer over this rank's CSR edge range, all-gathered to every rank."""
    nnz = engine.nnz
    if metric == "jaccard" and bounds is None and getattr(engine, "symmetric", False):
        return sharded_jaccard(engine, comm, out=kw.get("out"))
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


def sharded_sparsify(engine, comm: Comm, scores, num_edges: int, retention_ratio: float,
                     keep_lowest: bool = False, tie_break: str | None = None, out=None):
    """GraphSparsifier.sparsify's top-k (core.py:221-242) after the score
    all-gather: every rank holds the same full score vector (sharded_*), so every
    rank selects the same global top ``int(E*r)`` -- the radix select of
    gs_topk_mask on its own device, no further exchange.

    tie_break "stable": the device tie rule (= np.argsort(kind='stable'));
    "numpy": an ambiguous tie block at the cut is resolved by the reference's own
    np.argsort call on the host (identical on every rank of a node).  None (the
    default) resolves as GraphSparsifier does: $GSPARSE_TIE_BREAK, else "numpy" --
    so every rank keeps exactly the columns a single-GPU ``sparsify`` keeps.
    Returns (mask, info): a bool tensor on the comm device (a CPU tensor for gloo)
    and the cut / #beyond / #tied of the selection."""
    if not 0 < retention_ratio <= 1:
        raise ValueError(f"retention_ratio must be in (0, 1], got {retention_ratio}")
    import os

    tie_break = tie_break or os.environ.get("GSPARSE_TIE_BREAK", "numpy")
    if tie_break not in ("numpy", "stable"):
        raise ValueError(f"tie_break must be 'numpy' or 'stable', got {tie_break!r}")
    cuda = comm.device.type == "cuda"
    if retention_ratio == 1.0:
        m = torch.ones(num_edges, dtype=torch.bool, device=comm.device if cuda else "cpu")
        return m, {"cut": None, "beyond": num_edges, "tied": 0, "need": 0, "ambiguous": False}
    num_keep = int(num_edges * retention_ratio)
    if cuda:
        if out is None:
            out = torch.empty(num_edges, dtype=torch.uint8, device=comm.device)
        mask, cut, nb, nt = engine.topk_mask(scores, num_edges, num_keep, keep_lowest, out=out)
    else:
        s = scores.numpy() if isinstance(scores, torch.Tensor) else np.asarray(scores)
        m, cut, nb, nt = engine.topk_mask(s, num_edges, num_keep, keep_lowest)
        mask = torch.from_numpy(np.ascontiguousarray(m))
    need = num_keep - nb
    info = {"cut": cut, "beyond": nb, "tied": nt, "need": need, "ambiguous": 0 < need < nt}
    if info["ambiguous"] and tie_break == "numpy":
        from .selection import numpy_topk_mask

        s = scores.cpu().numpy() if isinstance(scores, torch.Tensor) else np.asarray(scores)
        m = torch.from_numpy(numpy_topk_mask(s, num_edges, num_keep, keep_lowest))
        mask = m.to(comm.device) if cuda else m
    return mask.view(torch.bool) if mask.dtype == torch.uint8 else mask, info


def _engine_device(engine) -> torch.device:
    ctx = getattr(engine, "ctx", None)
    return torch.device("cuda", ctx.device) if ctx is not None else torch.device("cpu")


def sharded_jaccard_topk(engine, comm: Comm, retention_ratio: float, keep_lowest: bool = False,
                         tie_break: str | None = None, mask_out=None, scores_out=None):
    """Jaccard-T over ranks (metrics.py:17-64 scores, then core.py:229-240's global top-k)
    without gathering the scores: every rank counts its owner pairs
    (gs_jaccard_part_counts), scores and keys them, and the ranks select the cut together
    by radix select over all-reduced histograms (gs_jsel_*: five passes, one SUM
    all-reduce of <= 64 KB each); an ambiguous tie block exchanges only its positions;
    each rank then sends a 2-bit keep code per own pair (an all-gather of ~E / 8 bytes in
    all) and every rank writes the whole CSR keep mask.

    The kept set equals a single GPU's ``sparsify`` on the same scores: the device tie
    rule (np.argsort(kind='stable')) for tie_break="stable"; for "numpy" (the default,
    $GSPARSE_TIE_BREAK) an ambiguous cut is resolved by the reference's own np.argsort on
    the gathered scores -- the only case that gathers them.  E = nnz (a symmetric graph's
    CSR entries; the bench's R-MAT).

    Returns (mask, info, scores): mask a uint8 tensor of nnz on the engine's device (or
    ``mask_out``), info the cut / #beyond / #tied / need / ambiguous, scores this rank's
    owner-pair scores (``scores_out`` if given; owner order of its row share)."""
    import os

    if not 0 < retention_ratio <= 1:
        raise ValueError(f"retention_ratio must be in (0, 1], got {retention_ratio}")
    tie_break = tie_break or os.environ.get("GSPARSE_TIE_BREAK", "numpy")
    if tie_break not in ("numpy", "stable"):
        raise ValueError(f"tie_break must be 'numpy' or 'stable', got {tie_break!r}")
    nnz = engine.nnz
    dev = _engine_device(engine)
    _, oo = engine.jaccard_shares(comm.world)
    sizes = np.diff(oo)
    stride = max(1, int(sizes.max()) if len(sizes) else 1)
    mine_pairs = int(sizes[comm.rank])
    counts = torch.zeros(stride, dtype=torch.int32, device=dev)
    if dev.type == "cuda":
        engine.jaccard_part_counts(comm.rank, comm.world, out=counts)
    else:
        part = np.asarray(engine.jaccard_part_counts(comm.rank, comm.world), dtype=np.uint32)
        counts[: part.shape[0]] = torch.from_numpy(part.view(np.int32))
    mask = mask_out if mask_out is not None else torch.empty(max(nnz, 1), dtype=torch.uint8, device=dev)
    num_keep = int(nnz * retention_ratio)
    if scores_out is None:
        scores_out = torch.empty(max(mine_pairs, 1), dtype=torch.float64, device=dev)
    if num_keep <= 0 or num_keep >= nnz:
        # nothing to select: idx[-0:] keeps all (top), idx[:0] none (keep_lowest)
        kept = not (keep_lowest and num_keep <= 0)
        mask[:nnz].fill_(1 if kept else 0)
        info = {"cut": None, "beyond": nnz if kept else 0, "tied": 0, "need": 0, "ambiguous": False}
        return mask, info, None

    def all_reduce(t):
        if t.device == comm.device:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=comm.group)
        else:
            c = t.to(comm.device)
            dist.all_reduce(c, op=dist.ReduceOp.SUM, group=comm.group)
            t.copy_(c)

    # device compute: the library's calls run without host waits (async: each call orders
    # the library's stream after torch's and torch's after the library's, so the RCCL
    # all-reduces in between see the histograms); only gs_jsel_result reads to the host
    ctx = getattr(engine, "ctx", None)
    go_async = ctx is not None and dev.type == "cuda" and not getattr(ctx, "_async", False)
    if go_async:
        ctx.set_async(True)
    try:
        return _jsel_select(engine, comm, dev, counts, stride, nnz, num_keep, keep_lowest, tie_break,
                            mask, scores_out, all_reduce)
    finally:
        if go_async:
            ctx.set_async(False)


def _jsel_select(engine, comm, dev, counts, stride, nnz, num_keep, keep_lowest, tie_break, mask,
                 scores_out, all_reduce):
    """sharded_jaccard_topk's select, after the counts (see there)."""
    hist = torch.zeros(engine.JSEL_BINS, dtype=torch.int64, device=dev)
    engine.jsel_begin(comm.rank, comm.world, counts, num_keep, keep_lowest, hist, scores_out)
    left = engine.JSEL_PASSES
    while left:
        all_reduce(hist)
        left = engine.jsel_step(hist)
    cut, nb, nt, my_tied = engine.jsel_result()
    need = num_keep - nb
    info = {"cut": cut, "beyond": nb, "tied": nt, "need": need, "ambiguous": 0 < need < nt}
    if info["ambiguous"] and tie_break == "numpy":
        from .selection import numpy_topk_mask

        s = sharded_jaccard(engine, comm)
        s = s.cpu().numpy() if isinstance(s, torch.Tensor) else np.asarray(s)
        m = torch.from_numpy(numpy_topk_mask(s, nnz, num_keep, keep_lowest).astype(np.uint8))
        mask[:nnz].copy_(m.to(mask.device))
        return mask, info, scores_out
    tie_all = None
    if info["ambiguous"]:
        cnt = comm.all_gather_same(torch.tensor([my_tied], dtype=torch.int64))
        tsz = [int(x.item()) for x in cnt]
        pos = torch.zeros(max(1, my_tied), dtype=torch.int64, device=dev)
        engine.jsel_tie_positions(pos)
        tie_all = comm.all_gather_padded(pos[:my_tied], tsz).to(dev)
        if tie_all.numel() != nt:
            raise RuntimeError(f"tie block: {tie_all.numel()} positions gathered, {nt} expected")
    stride4 = (stride + 3) // 4  # 2-bit codes, four pairs per byte
    keep = torch.zeros(stride4, dtype=torch.uint8, device=dev)
    engine.jsel_keep(tie_all, nt, need, keep)
    kall = comm.all_gather_flat(keep).to(dev)
    engine.jsel_mask(comm.world, kall, stride4, mask)
    return mask, info, scores_out


def backbone_phases(nbatch: int, world: int, fractions=None) -> list[tuple[int, int]]:
    """Search ranges of the staged backbone: batches [b0, b1) of the ascending-count
    order, cut at the given fractions of nbatch (default $GSPARSE_BB_PHASES, else
    BB_PHASES), one state exchange after each.  One rank: a single range."""
    import os

    if world <= 1 or nbatch == 0:
        return [(0, nbatch)]
    if fractions is None:
        env = os.environ.get("GSPARSE_BB_PHASES")
        fractions = ([float(x) for x in env.split(",") if x.strip()] if env
                     else BB_PHASES_4 if 4 <= world < 8 else BB_PHASES)
    cuts = sorted({int(round(f * nbatch)) for f in fractions if 0.0 < f < 1.0})
    bounds = [0] + [c for c in cuts if 0 < c < nbatch] + [nbatch]
    return list(zip(bounds[:-1], bounds[1:]))


# the ascending-count order's short searches decide most hub columns (reverse columns):
# the ranks exchange their decisions at these fractions of the batch list (RMAT-18, one
# rank's stages run alone, with the 3- / 4-edge local bounds: (0.6, 0.85) 251.5 / 150.3 /
# 105.0 ms at N = 2 / 4 / 8 against 407.6 ms whole; (0.7, 0.9) 262.5 / 161.1 / 108.8;
# (0.8) 258.2 / 145.7 / 110.6; tools/bb_stage_probe.py, profiles/r05z7_*)
BB_PHASES = (0.6, 0.85)
BB_PHASES_4 = (0.8,)  # 4 to 7 ranks


def sharded_backbone(comm: Comm, edge_index, num_nodes: int, edge_weights,
                     epsilon: float = 1e-9, stages=None, phases=None, keep_out=None,
                     method: str | None = None):
    """metric_backbone keep mask over ranks (metric_backbone.py:86-111), staged
    (include/gsparse.h gs_bb_*): every rank searches the landmarks l = rank (mod N)
    (MIN all-reduce of the labels), certifies its column range and searches its
    every N-th batch of each range of the ascending-count source order, with one
    MAX all-reduce of the E column-state bytes after each stage -- so a rank's later
    searches see every rank's earlier decisions (the short searches' reverse-column
    decisions close most hub columns before the hubs search).  Every rank returns
    the whole mask as a NumPy bool array, or fills `keep_out` (uint8, E entries, on
    the comm device) and returns it.

    `stages`: a BackboneStages (default: one on the library's shared context), or a
    stand-in with the same methods (the CPU tests).

    `method`: "staged" (above) or "pairs" -- the round-4 split: both directions of a
    pair decided by rank max(u, v) % N in one call (gs_metric_backbone_part), one SUM
    all-reduce of the keep bytes.  Default: "staged" (RMAT-18, a rank's work alone,
    before the 3- / 4-edge bounds: 276.6 vs 315.9 ms at N = 2, 116.7 vs 185.4 ms at
    N = 8; tools/bb_stage_probe.py, tools/bb_probe.py, profiles/r05u_*)."""
    from .metric_backbone import BackboneStages, check_weights

    E = (edge_index.shape[1] if not isinstance(edge_index, torch.Tensor)
         else int(edge_index.shape[1]))
    check_weights(edge_weights, E)
    st = stages if stages is not None else BackboneStages()
    if method is None:
        method = "staged"
    if method == "pairs":
        keep = keep_out if keep_out is not None else torch.empty(max(E, 1), dtype=torch.uint8,
                                                               device=comm.device)
        st.pair_part(edge_index, num_nodes, edge_weights, epsilon, comm.rank, comm.world, keep)
        if comm.world > 1 and E:
            dist.all_reduce(keep[:E], op=dist.ReduceOp.SUM, group=comm.group)
        if keep_out is not None:
            return keep_out
        return keep[:E].cpu().numpy().astype(bool)
    if method != "staged":
        raise ValueError(f"method must be 'staged' or 'pairs', got {method!r}")
    K = st.begin(edge_index, num_nodes, edge_weights, epsilon, comm.rank, comm.world)
    if comm.world > 1:
        # every rank must run the same schedule (the same number of collectives), whatever
        # its own environment says: K and the search ranges are checked / taken from rank 0
        agree = torch.tensor([K, -K], dtype=torch.int64, device=comm.device)
        dist.all_reduce(agree, op=dist.ReduceOp.MAX, group=comm.group)
        if int(agree[0]) != K or int(-agree[1]) != K:
            raise RuntimeError(f"ranks disagree on the landmark count (this rank {K}, range "
                               f"[{int(-agree[1])}, {int(agree[0])}]): set GSPARSE_BB_LANDMARKS alike")
    if K and comm.world > 1 and E and num_nodes:
        # rank r searched landmarks l = r (mod N) and holds only their labels (D is node-major,
        # D[u K + l]): each rank sends its own columns, every rank rebuilds the table
        n_ = int(num_nodes)
        D = torch.empty(K * n_, dtype=torch.float64, device=comm.device)
        comp = torch.empty(K, dtype=torch.int32, device=comm.device)
        st.landmarks_io(D, comp, out=True)
        per = (K + comm.world - 1) // comm.world
        mine = torch.arange(comm.rank, K, comm.world, device=comm.device)
        send = torch.full((n_, per), float("inf"), dtype=torch.float64, device=comm.device)
        send[:, : mine.numel()] = D.view(n_, K)[:, mine]
        got = comm.all_gather_flat(send.reshape(-1)).view(comm.world, n_, per)
        Dv = D.view(n_, K)
        for r in range(comm.world):
            cols = torch.arange(r, K, comm.world, device=comm.device)
            Dv[:, cols] = got[r, :, : cols.numel()]
        dist.all_reduce(comp, op=dist.ReduceOp.MAX, group=comm.group)
        st.landmarks_io(D, comp, out=False)
    st.certify(comm.rank, comm.world)
    state = torch.empty(max(E, 1), dtype=torch.uint8, device=comm.device)

    def exchange():
        if comm.world > 1 and E:
            st.state_io(state[:E], out=True)
            dist.all_reduce(state[:E], op=dist.ReduceOp.MAX, group=comm.group)
            st.state_io(state[:E], out=False)

    exchange()
    nb = st.plan()
    ranges = backbone_phases(nb, comm.world, phases)
    if comm.world > 1:  # rank 0's ranges ($GSPARSE_BB_PHASES / `phases` may differ per rank)
        cuts = torch.zeros(66, dtype=torch.int64, device=comm.device)
        if comm.rank == 0:
            if len(ranges) > 64:
                raise ValueError(f"at most 64 search ranges, got {len(ranges)}")
            cuts[0] = len(ranges)
            cuts[1: len(ranges) + 2] = torch.tensor([b for b, _ in ranges] + [nb], dtype=torch.int64)
        comm.broadcast_from(cuts, 0)
        k = int(cuts[0])
        b = [int(x) for x in cuts[1: k + 2]]
        ranges = list(zip(b[:-1], b[1:]))
    for b0, b1 in ranges:
        st.search(b0, b1, comm.rank, comm.world)
        exchange()
    keep = keep_out if keep_out is not None else torch.empty(max(E, 1), dtype=torch.uint8,
                                                           device=comm.device)
    st.finish(keep)
    if keep_out is not None:  # the caller's uint8 tensor, filled in place (bench: on the device)
        return keep_out
    return keep[:E].cpu().numpy().astype(bool)


def er_rank_blocks(k: int, world: int, max_depth: int = 5):
    """Column blocks of the pairwise tree of k for `world` ranks.

    Returns (depth, bounds, runs): the 2**depth nodes of the tree at `depth`
    (bounds, gs_er_split) and each rank's contiguous run [a, b) of them.  A
    power-of-two world takes one node per rank at depth log2(world); any other
    world the deepest level (<= max_depth, every node above it still split)
    with runs cut at the node boundaries nearest the equal column shares -- so
    every rank's columns are whole tree nodes whatever N is."""
    from .engine import er_split

    need = max(0, (world - 1).bit_length())
    top = need if world & (world - 1) == 0 else max(need, max_depth)
    # shallower levels when k is too small to split that far (some ranks idle)
    depths = list(range(top, -1, -1))
    for d in depths:
        try:
            bounds = er_split(k, 1 << d)
        except ValueError:
            continue
        # run boundaries at the node boundary nearest each rank's equal column share
        bnd = np.asarray(bounds)
        cut = [0] + [int(np.argmin(np.abs(bnd - k * r / world))) for r in range(1, world)] \
            + [len(bounds) - 1]
        for r in range(1, world + 1):
            cut[r] = max(cut[r], cut[r - 1])
        runs = [(cut[r], cut[r + 1]) for r in range(world)]
        return d, bounds, runs
    return 0, [0, k], [(0, 1)] + [(1, 1)] * (world - 1)


def dyadic_cover(a: int, b: int):
    """Maximal dyadic blocks (level, index) covering frontier nodes [a, b):
    level L block i spans nodes [i * 2**L, (i + 1) * 2**L) -- subtrees of the
    pairwise tree whose partial sums a rank can fold locally."""
    out = []
    while a < b:
        lev = 0
        while a % (2 << lev) == 0 and a + (2 << lev) <= b:
            lev += 1
        out.append((lev, a >> lev))
        a += 1 << lev
    return out


def sharded_approx_er(engine, comm: Comm, epsilon: float = 0.3, seed: int = 42,
                      max_cg_iters: int = 500, cg_tol: float = 1e-6, blas_threads: int = 1,
                      rng_mode: str = "device"):
    """ApproxER with the JL columns split over ranks along the pairwise tree."""
    from .engine import jl_dim

    n = engine.n
    k = jl_dim(n, epsilon)
    rng = np.random.default_rng(seed)
    m = engine.er_prepare(k)
    if m == 0:
        return comm.tensor(np.zeros(engine.nnz))
    depth, bounds, runs = er_rank_blocks(k, comm.world)
    a, b = runs[comm.rank]
    # this rank's JL columns only: the whole normal stream is parsed (it is sequential),
    # but only R[:, c0:c1] is stored and projected (metrics.py:272-275)
    cols = (bounds[a], bounds[b]) if b > a else (0, min(k, 1))
    if rng_mode == "device":
        engine.er_project_device(rng, k, cols=cols)
    else:
        engine.er_project_host(rng, k, cols=cols)
    covers = [dyadic_cover(a, b) for a, b in runs]
    cuda = comm.device.type == "cuda"
    dev = comm.device if cuda else "cpu"
    nnz = engine.nnz
    local = torch.zeros((max(1, len(covers[comm.rank])), nnz), dtype=torch.float64, device=dev)
    if b > a:
        engine.er_solve(bounds[a], bounds[b], max_cg_iters, cg_tol, blas_threads)
        for i, (lev, idx) in enumerate(covers[comm.rank]):
            lo, hi = idx << lev, (idx + 1) << lev

            def node_sums():  # the block's 2**lev nodes in tree order (gs_er_scores per node)
                for f in range(lo, hi):
                    o = torch.empty(nnz, dtype=torch.float64, device=comm.device) if cuda else None
                    p = engine.er_scores(bounds[f], bounds[f + 1], finalize=False, out=o)
                    yield p if cuda else torch.from_numpy(np.asarray(p))

            local[i] = fold_pairwise(node_sums())
    slots = [len(cv) for cv in covers]
    if all(sl == 1 for sl in slots):  # power-of-two world: one node per rank, one all-gather
        gathered = comm.all_gather_flat(local.reshape(-1)).reshape(comm.world, 1, nnz)
        blocks = [gathered[r] for r in range(comm.world)]
    else:  # every rank's real blocks only, from that rank
        blocks = [local if r == comm.rank else torch.empty((max(1, slots[r]), nnz), dtype=torch.float64,
                                                          device=dev)
                  for r in range(comm.world)]
        for r in range(comm.world):
            if slots[r]:
                comm.broadcast_from(blocks[r], r)
    level = {}
    for r, cv in enumerate(covers):
        for i, key in enumerate(cv):
            level[key] = blocks[r][i]
    for lev in range(depth):  # combine siblings bottom-up: the pairwise tree's own order
        for idx in range((1 << depth) >> (lev + 1)):
            lk, rk = (lev, 2 * idx), (lev, 2 * idx + 1)
            if lk in level and rk in level:
                level[(lev + 1, idx)] = level.pop(lk) + level.pop(rk)
    return finalize_er(level[(depth, 0)])
