"""CPU checks of the full-mask backbone fixtures (tests/golden/bb_rmat{16,17}.npz).

The GPU pins (tests/test_gpu_backbone_pins.py) compare the device mask with these
fixtures; here the fixture itself is re-derived in part: the R-MAT-16 graph and its
Jaccard costs hash to the stored digests, and the stored mask equals the oracle's
bounded Dijkstra (metric_backbone.py:86, 97-111 restated in oracle.c) on the hub rows
and a seeded sample of rows.  (The whole mask takes ~70 s on 8 threads:
tests/golden/make_backbone_fixtures.py.)
"""

from __future__ import annotations

import hashlib
import os

import numpy as np

import gsparse_oracle as O
from conftest import GOLDEN


def test_rmat16_backbone_fixture_rows_vs_oracle():
    from gsparse import graphs

    z = np.load(os.path.join(GOLDEN, "bb_rmat16.npz"), allow_pickle=False)
    n, E = int(z["n"]), int(z["E"])
    keep = np.unpackbits(z["keep_bits"])[:E].astype(bool)
    ei = graphs.rmat(16, 8, seed=0)
    assert ei.shape[1] == E and n == 1 << 16
    assert hashlib.sha256(ei.astype(np.int64).tobytes()).hexdigest() == str(z["edge_sha256"])
    ip, ix, _ = O.canonical_csr(ei, n)
    w = np.ascontiguousarray(O.scores_to_cost(O.jaccard(ip, ix), "jaccard")[:E])
    assert hashlib.sha256(w.tobytes()).hexdigest() == str(z["cost_sha256"])
    deg = np.diff(ip)
    rows = np.concatenate([np.argsort(deg, kind="stable")[-4:],
                           np.random.default_rng(16).choice(n, 512, replace=False)])
    ref, decided = O.metric_backbone_rows(ei, n, w, rows, threads=min(8, os.cpu_count() or 1))
    assert decided.sum() > 2000
    assert np.array_equal(keep[decided], ref[decided])
    assert 0 < keep.sum() < E


def test_rmat17_backbone_fixture_shape():
    z = np.load(os.path.join(GOLDEN, "bb_rmat17.npz"), allow_pickle=False)
    n, E = int(z["n"]), int(z["E"])
    keep = np.unpackbits(z["keep_bits"])[:E].astype(bool)
    assert n == 1 << 17 and keep.size == E and 0 < keep.sum() < E
    assert len(str(z["edge_sha256"])) == 64 and len(str(z["cost_sha256"])) == 64
