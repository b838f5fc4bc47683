"""Symmetric random baseline -- drop-in for ``src/sparsification/random.py``.

The result is defined by NumPy's ``default_rng(seed).random`` stream and
``np.unique``/``np.argsort`` (random.py:14-52); it is O(E) host work outside
the scoring hot path and is kept on the host unchanged.
"""

import numpy as np

from .data import Data


def precompute_random_scores(data: Data, seed: int = 42):
    """Reproducible symmetric random score per undirected edge (random.py:14-33)."""
    ei = data.edge_index.cpu().numpy()
    src, dst = ei[0], ei[1]
    n = data.num_nodes
    u = np.minimum(src, dst)
    v = np.maximum(src, dst)
    keys = u.astype(np.int64) * (n + 1) + v.astype(np.int64)
    _, inverse_idx = np.unique(keys, return_inverse=True)
    n_undirected = int(inverse_idx.max()) + 1
    rng = np.random.default_rng(seed)
    undirected_scores = rng.random(n_undirected)
    return undirected_scores, inverse_idx


def random_sparsify(data: Data, undirected_scores, inverse_idx, retention_ratio: float,
                    device: str) -> Data:
    """Keep the top fraction of undirected edges by random score (random.py:36-52)."""
    if retention_ratio == 1.0:
        return data.clone()
    n_undirected = len(undirected_scores)
    n_keep = max(1, int(n_undirected * retention_ratio))
    keep_undir = np.zeros(n_undirected, dtype=bool)
    keep_undir[np.argsort(undirected_scores)[-n_keep:]] = True
    mask = keep_undir[inverse_idx]
    sparse = data.clone()
    sparse.edge_index = data.edge_index[:, mask].to(device)
    return sparse
