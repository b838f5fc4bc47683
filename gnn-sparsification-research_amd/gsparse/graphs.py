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


def citation_like(n: int = 169_343, m: int = 1_166_243, seed: int = 0) -> np.ndarray:
    """Symmetrised citation graph of ogbn-arxiv size: exactly ``m`` distinct
    citations (ogbn-arxiv: 1,166,243 directed, one per undirected pair here, so
    2m = 2,332,486 CSR entries -- SURVEY 8(d)'s ~2.32M).

    Node s cites earlier nodes only (s > t): a uniform or a degree-biased target
    (the target of an earlier sampled citation, i.e. endpoint copying), each
    with probability 1/2.  Citation counts per node are fractional on average
    (m / (n - 1) = 6.89): every node cites floor(m / (n-1)), a seeded choice of
    the others one more; citations lost to duplicates are topped up by fresh
    draws (uniform citing node, same target rule) until exactly m remain."""
    if n < 2 or m < 0 or m > n * (n - 1) // 2:
        raise ValueError(f"citation_like: {m} distinct citations need 0 <= m <= n (n - 1) / 2 "
                         f"= {max(0, n * (n - 1) // 2)} (n = {n})")
    rng = np.random.default_rng(seed)
    nodes = np.arange(1, n, dtype=np.int64)
    base, extra = divmod(m, n - 1)
    per = np.full(n - 1, base, dtype=np.int64)
    per[rng.choice(n - 1, size=extra, replace=False)] += 1
    src = np.repeat(nodes, per)

    def targets(s: np.ndarray) -> np.ndarray:
        d = (rng.random(s.size) * s).astype(np.int64)  # uniform among earlier nodes
        copy = rng.random(s.size) < 0.5
        j = (rng.random(s.size) * np.arange(s.size)).astype(np.int64)
        return np.minimum(np.where(copy, d[j], d), s - 1)

    keys = np.unique(src * n + targets(src))
    rounds = 0
    while keys.size < m:
        # near the n (n - 1) / 2 limit fresh pairs get rare: bounded rounds, then a loud stop
        rounds += 1
        if rounds > 10_000:
            raise RuntimeError(f"citation_like: {keys.size} of {m} distinct citations after "
                               f"{rounds - 1} top-up rounds (m is too close to n (n - 1) / 2)")
        need = m - keys.size
        s = rng.integers(1, n, size=2 * need + 1024, dtype=np.int64)
        k = s * n + targets(s)
        k = k[~np.isin(k, keys)]
        _, first = np.unique(k, return_index=True)  # fresh keys, first draws in order
        keys = np.union1d(keys, k[np.sort(first)[:need]])
    return _symmetrise(keys // n, keys % n, n)


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
