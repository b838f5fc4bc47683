"""Full-mask pins of the metric backbone where every certificate class fires
("Next round" item 1; configs[4]).

* R-MAT-16 and R-MAT-17 with Jaccard costs (the bench's costs: _scores_to_cost of
  the device Jaccard, CSR order, the first E): the device keep mask equals the
  oracle's bounded Dijkstra over EVERY source row (``tests/golden/bb_rmat{16,17}.npz``,
  made by ``tests/golden/make_backbone_fixtures.py``) bit for bit -- with the default
  knobs, with the landmark certificates off (GSPARSE_BB_LANDMARKS=0), with the local
  bounds off (GSPARSE_BB_LOCALLB=0), and, on R-MAT-16, in the large-graph search
  geometry (16 sources per workgroup with reverse-column decisions).  R-MAT-17 is
  above the library's 65,536-node line, so it runs exactly the bench's R-MAT-18
  geometry (degree relabeling, 48 landmarks spread over the GPU, 16-source searches).
* The library records which exact rule decided each column (gs_bb_classes): the
  tests assert every class the verdict names fires on these graphs -- degree-1, the
  local bound, the 3-/4-edge bound, the 2-hop witness, landmark prune and the
  searches (keep and prune) with the default knobs; landmark keep with the local
  bounds off (they run first and take those columns otherwise); the reverse-column
  decisions in the large-graph geometry (R-MAT-17, and R-MAT-16 with 16 sources per
  workgroup) -- that every keeping rule keeps and every pruning rule prunes, and that
  no column is left without a class.
* R-MAT-18 (the bench's graph): >= 256 source rows stratified by decision class
  (up to 32 columns of each class that fired, plus the 8 hubs, plus random rows),
  every column of those rows against the oracle's per-row Dijkstra.

Reference: metric_backbone.py:86 (APSP), 97-111 (the per-column comparison).
"""

from __future__ import annotations

import contextlib
import hashlib
import os

import numpy as np
import pytest

import gsparse_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

# the classes VERDICT r05 asks to see fire (names of gsparse.metric_backbone.DECISION_CLASSES)
REQUIRED = ("landmark_keep", "landmark_prune", "degree1", "local_bound", "local_3_4_edge",
            "witness", "search_keep", "search_prune")
REVERSE = ("reverse_exact", "reverse_prune", "reverse_keep")


@contextlib.contextmanager
def _env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    try:
        for k, v in kv.items():
            os.environ[k] = str(v)
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _fixture(scale: int):
    z = np.load(os.path.join(GOLDEN, f"bb_rmat{scale}.npz"), allow_pickle=False)
    E = int(z["E"])
    keep = np.unpackbits(z["keep_bits"])[:E].astype(bool)
    return int(z["n"]), E, keep, str(z["edge_sha256"]), str(z["cost_sha256"])


def _device_costs(ei, n):
    """The bench's backbone costs from the device Jaccard (bit-exact vs the oracle)."""
    from gsparse._lib import Context
    from gsparse.engine import Engine

    ctx = Context(0)
    ctx.set_graph_edge_index(n, np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1]))
    jac = Engine(ctx).jaccard()
    return np.ascontiguousarray(O.scores_to_cost(jac, "jaccard")[: ei.shape[1]], dtype=np.float64)


@pytest.fixture(scope="module", params=[16, 17])
def rmat_case(request):
    from gsparse import graphs

    scale = request.param
    n, E, ref, edge_sha, cost_sha = _fixture(scale)
    ei = graphs.rmat(scale, 8, seed=0)
    assert ei.shape[1] == E and (1 << scale) == n
    assert _digest(ei.astype(np.int64)) == edge_sha  # the fixture's graph
    w = _device_costs(ei, n)
    assert _digest(w) == cost_sha  # the fixture's costs, bit for bit
    return scale, ei, n, w, ref


def _run(ei, n, w, **env):
    from gsparse.metric_backbone import backbone_mask, decision_classes, record_decision_classes

    with _env(**env):
        record_decision_classes(True)
        try:
            keep = backbone_mask(ei, n, w)
            counts, why = decision_classes(return_why=True)
        finally:
            record_decision_classes(False)
    return keep, counts, why


KNOBS = {
    "default": {},
    "no_landmarks": {"GSPARSE_BB_LANDMARKS": 0},
    "no_local_bounds": {"GSPARSE_BB_LOCALLB": 0},
    "no_certificates": {"GSPARSE_BB_LANDMARKS": 0, "GSPARSE_BB_LOCALLB": 0},
    # R-MAT-16 sits at the 65,536-node line: force the large-graph search geometry
    "multi16": {"GSPARSE_BB_MULTI": 16, "GSPARSE_BB_THREADS": 512},
}


@pytest.mark.parametrize("knobs", list(KNOBS))
def test_backbone_full_mask_vs_oracle_fixture(rmat_case, knobs):
    scale, ei, n, w, ref = rmat_case
    if knobs == "multi16" and scale != 16:
        pytest.skip("R-MAT-17 runs the large-graph geometry by default")
    keep, counts, why = _run(ei, n, w, **KNOBS[knobs])
    E = ei.shape[1]
    bad = np.flatnonzero(keep != ref)
    assert bad.size == 0, (knobs, bad.size, bad[:8].tolist())
    # every column carries the class of the rule that decided it
    assert counts["open"] == 0 and sum(counts.values()) == E, counts
    assert why.shape == (E,) and (why > 0).all()
    # class semantics: the pruning rules prune, the keeping rules keep
    from gsparse.metric_backbone import DECISION_CLASSES

    cls = {name: i for i, name in enumerate(DECISION_CLASSES)}
    for name in ("landmark_prune", "witness", "direct_edge", "reverse_prune"):
        assert not keep[why == cls[name]].any(), name
    for name in ("landmark_keep", "landmark_components", "local_bound", "local_3_4_edge",
                 "isolated", "reverse_keep"):
        assert keep[why == cls[name]].all(), name
    print(f"R-MAT-{scale} {knobs} decision classes:", {k: v for k, v in counts.items() if v})
    if knobs == "default":
        # with the local bounds on, they keep what a landmark lower bound would (they run
        # first): the landmark keeps fire with the local bounds off (below)
        for name in REQUIRED:
            if name != "landmark_keep":
                assert counts[name] > 0, (name, counts)
        if scale == 17:
            assert sum(counts[r] for r in REVERSE) > 0, counts
    if knobs == "no_local_bounds":
        assert counts["landmark_keep"] + counts["landmark_components"] > 0, counts
        assert counts["landmark_prune"] > 0 and counts["witness"] > 0, counts
    if knobs == "multi16":
        assert sum(counts[r] for r in REVERSE) > 0, counts
    if "GSPARSE_BB_LANDMARKS" in KNOBS[knobs]:
        assert counts["landmark_keep"] == counts["landmark_prune"] == counts["landmark_components"] == 0
    if "GSPARSE_BB_LOCALLB" in KNOBS[knobs]:
        assert counts["local_bound"] == counts["local_3_4_edge"] == counts["direct_edge"] == 0


def _host_threads() -> int:
    env = os.environ.get("OMP_NUM_THREADS")
    t = int(env) if env and env.isdigit() else (os.cpu_count() or 1)
    return max(1, min(16, t))


def test_backbone_rmat18_class_stratified_rows_vs_oracle():
    """configs[4]'s graph: >= 256 source rows chosen so every decision class that fired
    is represented (up to 32 columns per class), plus the 8 hubs and random rows; every
    column of those rows against the oracle's per-row Dijkstra (oracle.c)."""
    from gsparse import graphs
    from gsparse.metric_backbone import DECISION_CLASSES

    ei, n = graphs.rmat(18, 8, seed=0), 1 << 18
    w = _device_costs(ei, n)
    keep, counts, why = _run(ei, n, w)
    assert counts["open"] == 0
    src = ei[0]
    rng = np.random.default_rng(18)
    rows = []
    fired = [k for k in range(1, len(DECISION_CLASSES)) if counts[DECISION_CLASSES[k]] > 0]
    for k in fired:
        cols = np.flatnonzero(why == k)
        pick = rng.choice(cols, min(32, cols.size), replace=False)
        rows.append(src[pick])
    deg = np.bincount(src, minlength=n)
    rows.append(np.argsort(deg, kind="stable")[-8:])
    rows = np.unique(np.concatenate(rows))
    if rows.size < 256:
        rest = np.setdiff1d(np.arange(n), rows)
        rows = np.unique(np.concatenate([rows, rng.choice(rest, 256 - rows.size, replace=False)]))
    assert rows.size >= 256
    ref, decided = O.metric_backbone_rows(ei, n, w, rows, threads=_host_threads())
    for k in fired:  # every class is represented among the compared columns
        assert (decided & (why == k)).any(), DECISION_CLASSES[k]
    for name in REQUIRED:
        if name != "landmark_keep":  # the local bounds take those (see above)
            assert counts[name] > 0, (name, counts)
    assert sum(counts[r] for r in REVERSE) > 0, counts
    bad = np.flatnonzero(decided & (keep != ref))
    assert bad.size == 0, (bad.size, int(decided.sum()))
    print("R-MAT-18:", int(rows.size), "rows,", int(decided.sum()), "columns;",
          {k: v for k, v in counts.items() if v})
