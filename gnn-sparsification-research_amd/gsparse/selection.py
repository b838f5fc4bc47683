"""Host-side selection helpers whose results are DEFINED by NumPy calls.

``sparsify_sampled`` (core.py:333-350) is a draw from NumPy's
``Generator.choice`` stream and ``sparsify_degree_aware`` (core.py:415-453)
orders ties with ``np.argsort``; both are O(E) consumers of the device
scores kept on the host verbatim (SURVEY §8(f) rank 1 is their device port).
The functions take plain arrays so they are testable without a GPU.
"""

from __future__ import annotations

import numpy as np


def sampled_mask(scores: np.ndarray, num_edges: int, retention_ratio: float,
                 seed: int = 42) -> np.ndarray:
    """core.py:333-350 (the rng is created before the scores, as there)."""
    rng = np.random.default_rng(seed)
    floor = 1e-8
    s = np.nan_to_num(scores, nan=floor, posinf=floor, neginf=floor)
    probs = np.maximum(s, floor)
    probs = probs / probs.sum()
    num_keep = int(num_edges * retention_ratio)
    selected = rng.choice(num_edges, size=num_keep, replace=False, p=probs)
    mask = np.zeros(num_edges, dtype=bool)
    mask[selected] = True
    return mask


def degree_aware_mask(scores: np.ndarray, edge_index: np.ndarray, num_nodes: int,
                      num_edges: int, retention_ratio: float,
                      min_edges_per_node: int = 1) -> np.ndarray:
    """core.py:415-453 without the O(N*E) scans, same result.

    Phase 1: per node, ``incident[np.argsort(scores[incident])[-k:]]`` over its
    columns in ascending order (the reference's exact call is made whenever
    the pick is not unique: ties at the segment maximum, NaNs, or k > 1).
    Phase 2: the first non-guaranteed entries of ``np.argsort(scores)[::-1]``
    until ``int(E*r)`` columns are kept."""
    num_keep = int(num_edges * retention_ratio)
    src = np.asarray(edge_index)[0]
    order = np.argsort(src, kind="stable")
    bounds = np.searchsorted(src[order], np.arange(num_nodes + 1))
    counts = np.diff(bounds)
    mask = np.zeros(num_edges, dtype=bool)
    nonempty = np.nonzero(counts > 0)[0]
    exact_nodes = nonempty
    if min_edges_per_node == 1 and len(nonempty):
        sc = scores[order]  # IndexError when a column has no score, as the reference
        starts = bounds[nonempty]
        seg_max = np.maximum.reduceat(sc, starts)
        seg_id = np.repeat(np.arange(len(nonempty)), counts[nonempty])
        is_max = sc == seg_max[seg_id]
        n_max = np.bincount(seg_id, weights=is_max, minlength=len(nonempty))
        has_nan = np.bincount(seg_id, weights=np.isnan(sc), minlength=len(nonempty)) > 0
        unique = (n_max == 1) & ~has_nan
        pos = np.nonzero(is_max & unique[seg_id])[0]
        mask[order[pos]] = True
        exact_nodes = nonempty[~unique]
    for node in exact_nodes:
        lo, hi = bounds[node], bounds[node + 1]
        incident = order[lo:hi]
        k = min(min_edges_per_node, hi - lo)
        top_k = incident[np.argsort(scores[incident])[-k:]]
        mask[top_k] = True
    have = int(mask.sum())
    if have < num_keep:
        sorted_indices = np.argsort(scores)[::-1]
        cand = sorted_indices[~mask[sorted_indices]]
        mask[cand[: num_keep - have]] = True
    return mask


def degree_aware_mask_device(engine, scores: np.ndarray, edge_index: np.ndarray,
                             num_nodes: int, num_edges: int, retention_ratio: float,
                             min_edges_per_node: int = 1) -> np.ndarray:
    """degree_aware_mask with both phases on the MI355X; the same result.

    Phase 1: gs_segment_argmax gives every node's unique top column; nodes
    where np.argsort's order decides (ties at the maximum, NaN) take the
    reference's own call.  Phase 2: a device radix select over the scores with
    the guaranteed columns removed; an ambiguous tie block at the cut (or any
    NaN) takes the reference's own descending argsort walk."""
    scores = np.asarray(scores, dtype=np.float64)
    src = np.ascontiguousarray(np.asarray(edge_index)[0], dtype=np.int64)
    if min_edges_per_node != 1 or num_edges > len(scores) or np.isnan(scores).any():
        return degree_aware_mask(scores, edge_index, num_nodes, num_edges, retention_ratio,
                                 min_edges_per_node)
    num_keep = int(num_edges * retention_ratio)
    pick = engine.segment_argmax(scores, src[:num_edges], num_nodes)
    mask = np.zeros(num_edges, dtype=bool)
    mask[pick[pick >= 0]] = True
    amb = np.nonzero(pick == -2)[0]
    if len(amb):
        order = np.argsort(src, kind="stable")
        bounds = np.searchsorted(src[order], np.arange(num_nodes + 1))
        for node in amb:
            incident = order[bounds[node]:bounds[node + 1]]
            mask[incident[np.argsort(scores[incident])[-1:]]] = True
    have = int(mask.sum())
    if have >= num_keep:
        return mask
    k2 = num_keep - have
    masked = scores.copy()
    masked[np.nonzero(mask)[0]] = -np.inf
    sel, cut, beyond, tied = engine.topk_mask(masked, num_edges, k2, False)
    need = k2 - beyond
    if (0 < need < tied) or cut == -np.inf:
        # the reference's own walk: first non-guaranteed of argsort(scores)[::-1]
        sorted_indices = np.argsort(scores)[::-1]
        cand = sorted_indices[~mask[sorted_indices]]
        mask[cand[:k2]] = True
        return mask
    return mask | sel


def numpy_topk_mask(scores: np.ndarray, num_edges: int, num_keep: int,
                    keep_lowest: bool) -> np.ndarray:
    """core.py:233-240 verbatim: the reference's unstable argsort tie order."""
    idx = np.argsort(scores)
    sel = idx[:num_keep] if keep_lowest else idx[-num_keep:]
    mask = np.zeros(num_edges, dtype=bool)
    mask[sel] = True
    return mask
