"""Global metric backbone -- drop-in for ``src/sparsification/metric_backbone.py``.

``compute_metric_backbone`` keeps column (u,v) of ``edge_index`` iff
w_uv <= d_G(u,v) + epsilon (or d is infinite), with G the undirected graph of
the u<v columns (metric_backbone.py:28-141).  The reference runs NetworkX
all-pairs Dijkstra into an O(n^2) dict; here libgsparse resolves each column
with an exact 2-hop witness test and, where that is inconclusive, an exact
bounded shortest-path search from u on the MI355X (gs_metric_backbone) --
the same distances bit for bit, no APSP table.
"""

from __future__ import annotations

import ctypes
from typing import Dict, Tuple

import numpy as np
import torch
from numpy.typing import NDArray

from ._lib import GS_HOST, Context, ptr
from .data import Data

_CTX = None


def _context(ctx: Context | None) -> Context:
    global _CTX
    if ctx is not None:
        return ctx
    if _CTX is None:
        _CTX = Context()
    return _CTX


def check_weights(edge_weights, n_edges: int) -> None:
    """The reference reads ``edge_weights[idx]`` for every edge_index column
    (metric_backbone.py:73-74): fewer weights than columns is NumPy's
    IndexError there, and must never reach the library as a short buffer."""
    nw = len(edge_weights)
    if nw < n_edges:
        raise IndexError(f"index {nw} is out of bounds for axis 0 with size {nw}")


def backbone_mask(edge_index: np.ndarray, num_nodes: int, edge_weights: np.ndarray,
                  epsilon: float = 1e-9, ctx: Context | None = None,
                  return_relax: bool = False, part: int = 0, nparts: int = 1):
    """Keep mask (bool[E]) of the metric backbone; device computation.

    With nparts > 1 only the columns (u, v) with max(u, v) % nparts == part (ids
    as the library labels them: graphs without id locality are relabeled by
    degree first) are decided here (the rest read False): the parts OR to the
    whole mask."""
    ei = np.asarray(edge_index, dtype=np.int64)
    E = ei.shape[1]
    src = np.ascontiguousarray(ei[0])
    dst = np.ascontiguousarray(ei[1])
    w = np.ascontiguousarray(np.asarray(edge_weights, dtype=np.float64).reshape(-1)[:E])
    check_weights(w, E)
    keep = np.zeros(max(E, 1), dtype=np.uint8)
    relax = ctypes.c_int64(0)
    c = _context(ctx)
    c.call("gs_metric_backbone_part", int(num_nodes), E, ptr(src), ptr(dst), ptr(w), len(w),
           GS_HOST, float(epsilon), int(part), int(nparts), ptr(keep), GS_HOST,
           ctypes.byref(relax))
    mask = keep[:E].view(bool)
    return (mask, relax.value) if return_relax else mask


class BackboneStages:
    """The staged prune on one context (gs_bb_*, include/gsparse.h): what one rank of
    ``gsparse.distributed.sharded_backbone`` runs between its exchanges.  Array
    arguments are NumPy arrays / CPU tensors (host) or device tensors.

    The library reads 8 B per column of src / dst / weights and writes 1 B per column
    of keep / state, so every buffer is checked here before its pointer is taken:
    columns and weights are cast to int64 / float64 (copies, kept alive for the run),
    output buffers must already be uint8 (resp. float64 / int32 landmark buffers) and
    large enough, and device tensors must live on the context's device."""

    def __init__(self, ctx: Context | None = None):
        self.ctx = _context(ctx)
        self.n = self.E = self.K = 0

    @staticmethod
    def _p(a):
        from ._lib import GS_DEVICE

        if isinstance(a, torch.Tensor):
            return a.data_ptr(), (GS_DEVICE if a.is_cuda else GS_HOST)
        return ptr(a), GS_HOST

    def _on_device(self, t: torch.Tensor, what: str) -> None:
        if t.is_cuda and t.device.index != self.ctx.device:
            raise ValueError(f"{what} is on {t.device}, the context drives cuda:{self.ctx.device}")

    def _out(self, buf, dtype, count: int, what: str):
        """An output buffer the library writes `count` elements of `dtype` into."""
        if isinstance(buf, torch.Tensor):
            tdt = {np.uint8: torch.uint8, np.float64: torch.float64, np.int32: torch.int32}[dtype]
            if buf.dtype != tdt:
                raise TypeError(f"{what} must be {tdt}, got {buf.dtype}")
            if not buf.is_contiguous():
                raise ValueError(f"{what} must be contiguous")
            self._on_device(buf, what)
            n = buf.numel()
        else:
            if not isinstance(buf, np.ndarray) or buf.dtype != dtype or not buf.flags.c_contiguous:
                raise TypeError(f"{what} must be a contiguous {np.dtype(dtype)} array")
            n = buf.size
        if n < count:
            raise ValueError(f"{what} holds {n} entries, the library writes {count}")
        return self._p(buf)

    def _columns(self, edge_index, edge_weights):
        """(src, dst, w) as int64 / int64 / float64 on one side, E, and their pointers."""
        if isinstance(edge_index, torch.Tensor) and edge_index.is_cuda:
            self._on_device(edge_index, "edge_index")
            if edge_index.dim() != 2 or edge_index.shape[0] != 2:
                raise ValueError("edge_index must be [2, E]")
            src = edge_index[0].to(torch.int64).contiguous()
            dst = edge_index[1].to(torch.int64).contiguous()
            E = int(src.numel())
        else:
            ei = np.asarray(edge_index.cpu() if isinstance(edge_index, torch.Tensor) else edge_index,
                            dtype=np.int64)
            E = ei.shape[1]
            src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
        if isinstance(edge_weights, torch.Tensor) and edge_weights.is_cuda:
            self._on_device(edge_weights, "edge_weights")
            w = edge_weights.reshape(-1)[:E].to(torch.float64).contiguous()
        else:
            ew = edge_weights.cpu() if isinstance(edge_weights, torch.Tensor) else edge_weights
            w = np.ascontiguousarray(np.asarray(ew, dtype=np.float64).reshape(-1)[:E])
        check_weights(w, E)
        (ps, loc), (pd, _), (pw, wloc) = self._p(src), self._p(dst), self._p(w)
        if loc != wloc:
            raise ValueError("edge_index and edge_weights must be on the same side")
        self._keep_alive = (src, dst, w)
        return E, ps, pd, pw, len(w), loc

    def begin(self, edge_index, num_nodes: int, edge_weights, epsilon: float, part: int,
              nparts: int) -> int:
        """Graph, columns by row, landmark searches l = part (mod nparts); returns K."""
        E, ps, pd, pw, nw, loc = self._columns(edge_index, edge_weights)
        K = ctypes.c_int32(0)
        self.ctx.call("gs_bb_begin", int(num_nodes), E, ps, pd, pw, nw, loc, float(epsilon),
                      int(part), int(nparts), ctypes.byref(K))
        self.n, self.E, self.K = int(num_nodes), E, int(K.value)
        return self.K

    def pair_part(self, edge_index, num_nodes: int, edge_weights, epsilon: float, part: int,
                  nparts: int, keep):
        """gs_metric_backbone_part: keep bytes of the columns (u, v) with max(u, v) %
        nparts == part (ids as the library labels them), 0 elsewhere, into `keep`."""
        E, ps, pd, pw, nw, loc = self._columns(edge_index, edge_weights)
        pk, kloc = self._out(keep, np.uint8, max(E, 1), "keep")
        relax = ctypes.c_int64(0)
        self.ctx.call("gs_metric_backbone_part", int(num_nodes), E, ps, pd, pw, nw, loc,
                      float(epsilon), int(part), int(nparts), pk, kloc, ctypes.byref(relax))
        self.relax = relax.value
        return keep

    def landmarks_io(self, D, complete, out: bool):
        if self.K == 0 or self.E == 0:
            return  # the library copies nothing then
        pD, loc = self._out(D, np.float64, self.K * self.n, "landmark labels D")
        pc, cloc = self._out(complete, np.int32, self.K, "landmark completeness flags")
        if loc != cloc:
            raise ValueError("D and complete must be on the same side")
        self.ctx.call("gs_bb_landmarks_io", pD, pc, loc, 0 if out else 1)

    def certify(self, part: int, nparts: int):
        self.ctx.call("gs_bb_certify", int(part), int(nparts))

    def state_io(self, state, out: bool):
        if self.E == 0:
            return
        p, loc = self._out(state, np.uint8, self.E, "state")
        self.ctx.call("gs_bb_state_io", p, loc, 0 if out else 1)

    def plan(self) -> int:
        nb = ctypes.c_int64(0)
        self.ctx.call("gs_bb_plan", ctypes.byref(nb))
        return int(nb.value)

    def search(self, b0: int, b1: int, part: int, nparts: int):
        self.ctx.call("gs_bb_search", int(b0), int(b1), int(part), int(nparts))

    def finish(self, keep=None):
        """Keep bytes of every column (into ``keep`` if given) and the relaxations."""
        if keep is None:
            keep = np.zeros(max(self.E, 1), dtype=np.uint8)
        p, loc = self._out(keep, np.uint8, max(self.E, 1), "keep")
        relax = ctypes.c_int64(0)
        self.ctx.call("gs_bb_finish", p, loc, ctypes.byref(relax))
        self._keep_alive = None
        self.relax = relax.value
        return keep, relax.value


#: decision classes of gs_bb_class_counts (include/gsparse.h GS_BB_WHY_*)
DECISION_CLASSES = ("open", "self_loop", "isolated", "degree1", "direct_edge", "local_bound",
                    "landmark_components", "landmark_prune", "landmark_keep", "witness",
                    "local_3_4_edge", "search_prune", "search_keep", "reverse_exact",
                    "reverse_prune", "reverse_keep", "meet_in_middle")


def record_decision_classes(on: bool = True, ctx: Context | None = None) -> None:
    """Make the following backbone runs on ``ctx`` record which exact rule decided each
    column (gs_bb_classes; a diagnostic for the parity tests)."""
    _context(ctx).call("gs_bb_classes", 1 if on else 0)


def decision_classes(ctx: Context | None = None, return_why: bool = False):
    """Columns per decision class of the last backbone run on ``ctx`` (this rank's
    decisions), as {class name: count}; with return_why also the per-column class bytes
    (uint8[E], indices into DECISION_CLASSES)."""
    c = _context(ctx)
    counts = np.zeros(len(DECISION_CLASSES), dtype=np.int64)
    E = ctypes.c_int64(0)
    c.call("gs_bb_class_counts", ptr(counts), len(counts), None, 0, GS_HOST, ctypes.byref(E))
    out = {name: int(v) for name, v in zip(DECISION_CLASSES, counts)}
    if not return_why:
        return out
    why = np.zeros(max(E.value, 1), dtype=np.uint8)
    c.call("gs_bb_class_counts", ptr(counts), len(counts), ptr(why), why.size, GS_HOST, None)
    return out, why[: E.value]


def compute_metric_backbone(
    data: Data,
    edge_weights: NDArray[np.float64],
    epsilon: float = 1e-9,
    verbose: bool = True,
    _ctx: Context | None = None,
) -> Tuple[Data, Dict]:
    """Compute the Global Metric Backbone (metric_backbone.py:28-141).

    Returns ``(sparsified_data, stats)`` with the reference's stats keys."""
    edge_index = data.edge_index.cpu().numpy()
    rows = edge_index[0]
    n_nodes = data.num_nodes
    n_edges = len(rows)

    if verbose:
        print(f"Computing Global Metric Backbone")
        print(f"  Nodes: {n_nodes:,}, Edges: {n_edges:,}")
        print(f"  Epsilon: {epsilon}")

    edge_weights = np.asarray(edge_weights)
    check_weights(edge_weights, n_edges)
    if verbose:
        m = rows < edge_index[1]
        und = len(np.unique(rows[m].astype(np.int64) * max(n_nodes, 1) + edge_index[1][m]))
        print(f"  Unique undirected edges: {und:,}")
        print(f"  Computing APSP via Dijkstra... ", end="", flush=True)

    keep_mask = backbone_mask(edge_index, n_nodes, edge_weights, epsilon, _ctx)

    if verbose:
        print("Done!")
        print(f"  Classifying edges...")

    edges_metric = int(keep_mask.sum())
    edges_semi_metric = n_edges - edges_metric
    sparse_edge_index = torch.from_numpy(edge_index[:, keep_mask])
    sparse_data = data.clone()
    sparse_data.edge_index = sparse_edge_index
    sparse_weights = edge_weights[keep_mask] if len(edge_weights) == n_edges else \
        edge_weights[:n_edges][keep_mask]

    stats = {
        "original_edges": n_edges,
        "retained_edges": int(keep_mask.sum()),
        "removed_edges": int((~keep_mask).sum()),
        "retention_ratio": float(keep_mask.sum() / n_edges),
        "edges_metric": edges_metric,
        "edges_semi_metric": edges_semi_metric,
        "epsilon": epsilon,
        "sparse_weights": sparse_weights,
        "keep_mask": keep_mask,
    }

    if verbose:
        print(f"\n{'='*50}")
        print(f"Metric Backbone Results")
        print(f"{'='*50}")
        print(f"  Original edges:        {stats['original_edges']:,}")
        print(
            f"  Metric (retained):     {stats['retained_edges']:,} ({stats['retention_ratio']:.1%})"
        )
        print(f"  Semi-metric (removed): {stats['removed_edges']:,}")

    return sparse_data, stats


def pair_distances(edge_index: np.ndarray, num_nodes: int, weights, pairs,
                   ctx: Context | None = None) -> np.ndarray:
    """Exact shortest-path distances (+inf if unreachable) between node pairs in
    the graph metric_backbone.py:70-79 builds (gs_pair_distances); weights None:
    hop counts."""
    c = _context(ctx)
    ei = np.asarray(edge_index, dtype=np.int64)
    src = np.ascontiguousarray(ei[0])
    dst = np.ascontiguousarray(ei[1])
    w = None
    if weights is not None:
        w = np.ascontiguousarray(np.asarray(weights, dtype=np.float64).reshape(-1)[: ei.shape[1]])
        check_weights(w, ei.shape[1])
    pr = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    qs = np.ascontiguousarray(pr[:, 0])
    qt = np.ascontiguousarray(pr[:, 1])
    out = np.empty(len(pr), dtype=np.float64)
    c.call("gs_pair_distances", int(num_nodes), int(ei.shape[1]), ptr(src), ptr(dst),
           ptr(w) if w is not None else None, 0 if w is None else len(w), GS_HOST, int(len(pr)),
           ptr(qs), ptr(qt), ptr(out))
    return out


def verify_geodesic_preservation(
    original_data: Data,
    sparse_data: Data,
    original_weights: NDArray[np.float64],
    sparse_weights: NDArray[np.float64],
    n_samples: int = 500,
    epsilon: float = 1e-6,
    seed: int = 42,
) -> Dict:
    """Verify that the Metric Backbone preserves geodesic distances
    (metric_backbone.py:144-225): the same sampled pairs (the reference's RNG
    calls), the same weighted graphs (u < v columns, minimum weight over
    duplicates), distances from gs_pair_distances -- exact searches, equal to
    NetworkX's Dijkstra bit for bit -- and the same bookkeeping."""
    rng = np.random.default_rng(seed)
    n = original_data.num_nodes
    pairs = set()
    while len(pairs) < n_samples:
        u, v = rng.integers(0, n, size=2)
        if u != v:
            pairs.add((min(u, v), max(u, v)))
    pairs = list(pairs)
    ei_o = original_data.edge_index.cpu().numpy()
    ei_s = sparse_data.edge_index.cpu().numpy()
    d_o = pair_distances(ei_o, n, original_weights, pairs)
    d_s = pair_distances(ei_s, sparse_data.num_nodes, sparse_weights, pairs)
    violations = []
    verified = 0
    unreachable_original = 0
    unreachable_backbone = 0
    for (u, v), a, b in zip(pairs, d_o, d_s):
        if np.isinf(a):
            unreachable_original += 1
            continue
        d_orig = float(a)
        if np.isinf(b):
            unreachable_backbone += 1
            violations.append((u, v, d_orig, float("inf"), float("inf")))
            continue
        d_back = float(b)
        diff = abs(d_orig - d_back)
        if diff > epsilon:
            violations.append((u, v, d_orig, d_back, diff))
        else:
            verified += 1
    return {
        "pairs_tested": len(pairs),
        "verified_equal": verified,
        "violations": len(violations),
        "unreachable_original": unreachable_original,
        "unreachable_backbone": unreachable_backbone,
        "max_violation": max([v[4] for v in violations]) if violations else 0.0,
        "geodesic_preserved": len(violations) == 0,
        "violation_details": violations[:5],
    }
