"""Deterministic synthetic graphs standing in for the reference's datasets.

The reference loads Cora / Roman-empire / ogbn-arxiv through a PyG
downloader (``src/data``, absent from the snapshot) — there is no network
here, so every benchmark and parity case runs on the synthetic stand-ins
specified in SURVEY.md §8(d).  All generators return an ``edge_index`` of
shape ``[2, E]`` (int64, numpy) that is symmetric, duplicate-free, loop-free
and row-major sorted — i.e. the layout PyG's coalesced datasets have, which
is the layout under which the reference's CSR-ordered scores and its
edge_index-ordered masks agree (SURVEY.md §0 finding 4).
"""

from __future__ import annotations

import numpy as np


def _symmetrise(u: np.ndarray, v: np.ndarray, n: int) -> np.ndarray:
    """Undirected pairs -> sorted, deduplicated, loop-free directed edge_index."""
    u = np.asarray(u, dtype=np.int64)
    v = np.asarray(v, dtype=np.int64)
    keep = u != v
    u, v = u[keep], v[keep]
    src = np.concatenate([u, v])
    dst = np.concatenate([v, u])
    keys = np.unique(src * n + dst)
    return np.stack([keys // n, keys % n]).astype(np.int64)


def roman_like(n: int = 22_662, m: int = 32_927, seed: int = 0) -> np.ndarray:
    """Chain 0..n-1 plus short-range chords (a, a+1+Geom(0.3)).

    Roman-empire (Platonov et al.) is a word-adjacency chain with a few
    syntactic chords; its size is n=22,662, 32,927 undirected edges.
    """
    if m < n - 1:
        raise ValueError("m must cover the path")
    rng = np.random.default_rng(seed)
    path = np.arange(n - 1, dtype=np.int64)
    keys = set((path * n + path + 1).tolist())
    need = m - (n - 1)
    chords_u, chords_v = [], []
    while need > 0:
        a = rng.integers(0, n, size=4 * need + 64)
        gap = 1 + rng.geometric(0.3, size=a.size)
        b = a + gap
        for x, y in zip(a.tolist(), b.tolist()):
            if y >= n:
                continue
            k = x * n + y
            if k in keys:
                continue
            keys.add(k)
            chords_u.append(x)
            chords_v.append(y)
            need -= 1
            if need == 0:
                break
    u = np.concatenate([path, np.asarray(chords_u, dtype=np.int64)])
    v = np.concatenate([path + 1, np.asarray(chords_v, dtype=np.int64)])
    return _symmetrise(u, v, n)


def rmat(scale: int, edge_factor: int = 8, seed: int = 0,
         abc: tuple = (0.57, 0.19, 0.19)) -> np.ndarray:
    """Graph500 R-MAT: 2^scale nodes, edge_factor*2^scale samples.

    Vertex labels are randomly permuted, self-loops dropped, the result is
    symmetrised and deduplicated.
    """
    n = 1 << scale
    ne = edge_factor * n
    a, b, c = abc
    rng = np.random.default_rng(seed)
    src = np.zeros(ne, dtype=np.int64)
    dst = np.zeros(ne, dtype=np.int64)
    chunk = 1 << 22
    for lo in range(0, ne, chunk):
        hi = min(ne, lo + chunk)
        s = np.zeros(hi - lo, dtype=np.int64)
        d = np.zeros(hi - lo, dtype=np.int64)
        for lvl in range(scale):
            r = rng.random(hi - lo)
            sbit = r >= a + b
            dbit = ((r >= a) & (r < a + b)) | (r >= a + b + c)
            s |= sbit.astype(np.int64) << lvl
            d |= dbit.astype(np.int64) << lvl
        src[lo:hi] = s
        dst[lo:hi] = d
    perm = rng.permutation(n).astype(np.int64)
    return _symmetrise(perm[src], perm[dst], n)


def chung_lu(n: int = 2_708, m: int = 5_278, gamma: float = 2.5, seed: int = 0) -> np.ndarray:
    """Power-law (Chung-Lu) graph with exactly m undirected edges (Cora stand-in)."""
    rng = np.random.default_rng(seed)
    w = (np.arange(1, n + 1, dtype=np.float64)) ** (-1.0 / (gamma - 1.0))
    p = w / w.sum()
    keys: set = set()
    us, vs = [], []
    while len(keys) < m:
        a = rng.choice(n, size=2 * m, p=p)
        b = rng.choice(n, size=2 * m, p=p)
        for x, y in zip(a.tolist(), b.tolist()):
            if x == y:
                continue
            if x > y:
                x, y = y, x
            k = x * n + y
            if k in keys:
                continue
            keys.add(k)
            us.append(x)
            vs.append(y)
            if len(keys) == m:
                break
    perm = rng.permutation(n)
    return _symmetrise(perm[np.asarray(us)], perm[np.asarray(vs)], n)


def citation_like(n: int = 169_343, m: int = 1_160_000, seed: int = 0) -> np.ndarray:
    """Symmetrised preferential-attachment-style graph of ogbn-arxiv size."""
    rng = np.random.default_rng(seed)
    # Each node cites ~m/n earlier nodes, chosen by a mix of uniform and
    # degree-biased (via endpoint copying) selection.
    per = max(1, m // n)
    src = np.repeat(np.arange(1, n, dtype=np.int64), per)
    u = rng.random(src.size)
    dst = (u * src).astype(np.int64)  # uniform among earlier nodes
    copy = rng.random(src.size) < 0.5
    # degree bias: copy the target of an earlier sampled edge
    j = (rng.random(src.size) * np.arange(src.size)).astype(np.int64)
    dst = np.where(copy, dst[j], dst)
    dst = np.minimum(dst, src - 1)
    return _symmetrise(src, dst, n)


def features(n: int, f: int, seed: int = 1, kind: str = "normal") -> np.ndarray:
    """float32 node features: N(0,1) or Bernoulli(p) bag-of-words."""
    rng = np.random.default_rng(seed)
    if kind == "normal":
        return rng.standard_normal((n, f), dtype=np.float32)
    if kind == "bow":
        return (rng.random((n, f)) < 0.0127).astype(np.float32)
    raise ValueError(kind)


def karate(order: str = "test") -> tuple[np.ndarray, int]:
    """Zachary karate club as the reference's tests build it.

    order="test": ``[edges] + [reversed edges]`` (tests/test_sparsification.py:33-42),
    which is NOT row-major; order="csr": the same edge set sorted.
    """
    import networkx as nx

    g = nx.karate_club_graph()
    el = list(g.edges())
    ei = np.array([[u, v] for u, v in el] + [[v, u] for u, v in el], dtype=np.int64).T
    if order == "csr":
        n = g.number_of_nodes()
        keys = np.sort(ei[0] * n + ei[1])
        ei = np.stack([keys // n, keys % n])
    return np.ascontiguousarray(ei), g.number_of_nodes()
