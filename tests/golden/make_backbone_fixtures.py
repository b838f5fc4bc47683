"""Full keep masks of the metric backbone on R-MAT-16 / -17 with Jaccard costs (fixtures).

    python tests/golden/make_backbone_fixtures.py            # R-MAT-16, ~70 s on 8 threads
    python tests/golden/make_backbone_fixtures.py --scale 17 # R-MAT-17, ~5 min

The graph is ``gsparse.graphs.rmat(S, 8, seed=0)`` (S = 16: n = 65,536, E = 955,124;
S = 17: n = 131,072, the library's large-graph geometry, as the bench's R-MAT-18); its
costs are the bench's: ``_scores_to_cost(jaccard)`` in CSR order, the first E
(core.py:82-116 applied to metrics.py:17-64's scores, restated by the oracle).  The
mask is the oracle's bounded Dijkstra of every source row (``oracle.c``, the
restatement of metric_backbone.py:86 / 97-111 that ``tests/test_oracle_golden.py``
pins to the reference's own NetworkX APSP on the golden graphs).  NetworkX APSP
itself would take hours at this size, so the fixture is the pinned oracle's output.

Stored (no reference source, vectors only): the packed keep mask, n, E, and SHA-256
digests of the edge_index bytes and of the cost bytes, so a test that regenerates
the graph and its costs can prove it has the same inputs before comparing masks.
"""

from __future__ import annotations

import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "gnn-sparsification-research_amd"), os.path.join(REPO, "oracle")]

import gsparse_oracle as O  # noqa: E402
from gsparse import graphs  # noqa: E402

EDGE_FACTOR, SEED = 8, 0


def inputs(scale: int = 16):
    """(edge_index, n, costs) of the fixture."""
    ei, n = graphs.rmat(scale, EDGE_FACTOR, seed=SEED), 1 << scale
    ip, ix, _ = O.canonical_csr(ei, n)
    w = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")[: ei.shape[1]]
    return ei, n, np.ascontiguousarray(w, dtype=np.float64)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=16)
    scale = ap.parse_args().scale
    t0 = time.time()
    ei, n, w = inputs(scale)
    E = ei.shape[1]
    threads = min(16, os.cpu_count() or 1)
    keep, decided = O.metric_backbone_rows(ei, n, w, np.arange(n), threads=threads)
    assert decided.all()
    out = os.path.join(HERE, f"bb_rmat{scale}.npz")
    np.savez_compressed(out, n=np.int64(n), E=np.int64(E), keep_bits=np.packbits(keep),
                        edge_sha256=np.array(digest(ei.astype(np.int64))),
                        cost_sha256=np.array(digest(w)), scale=np.int64(scale),
                        edge_factor=np.int64(EDGE_FACTOR), seed=np.int64(SEED))
    print(f"{out}: n={n} E={E} kept={int(keep.sum())} in {time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
