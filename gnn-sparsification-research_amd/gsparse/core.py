"""GraphSparsifier -- drop-in for ``src/sparsification/core.py``.

Same class name, constructor, attributes (``data, device, num_nodes,
num_edges, adj, verbose, _score_cache, SUPPORTED_METRICS,
_DISTANCE_METRICS``), methods and error behaviour as the reference
(core.py:24-490).  The canonical CSR is built on the MI355X and stays
resident there for every scorer; ``adj`` (a SciPy CSR) is materialised on
first access.  ``SparsificationEngine`` is an alias (BASELINE north_star name).

Selection semantics (core.py:229-242): the device top-k keeps exactly the
``int(E*r)`` highest (lowest) CSR-ordered scores.  Edges strictly beyond the
cut are identical to the reference by construction.  Inside a tie block at
the cut the reference's ``np.argsort`` (unstable, SIMD-dispatch dependent)
decides; ``tie_break="numpy"`` (default, the drop-in behaviour) resolves an
ambiguous tie block with that very call on the host, ``tie_break="stable"``
keeps the device rule (= ``np.argsort(kind="stable")``).
"""

from __future__ import annotations

import os
from typing import Dict, Tuple

import numpy as np
import scipy.sparse as sp
import torch

from ._lib import Context
from .data import Data
from .engine import Engine
from .metric_backbone import compute_metric_backbone
from .selection import degree_aware_mask_device, numpy_topk_mask, sampled_mask


def _device_index(device) -> int | None:
    s = str(device)
    if s.startswith("cuda:"):
        try:
            return int(s.split(":", 1)[1])
        except ValueError:
            return None
    return None


class GraphSparsifier:
    """Engine for graph sparsification via edge metric thresholding.

    Args:
        data: PyG ``Data`` (or ``gsparse.Data``) with ``edge_index`` [2, E].
        device: where returned graphs are placed (as in the reference).
        tie_break: "numpy" (default) or "stable", see module docstring.
        gpu: libgsparse device ordinal (default: cuda:N of ``device``,
            else $GSPARSE_DEVICE / $LOCAL_RANK / 0).
    """

    SUPPORTED_METRICS = {
        "jaccard",
        "adamic-adar",
        "adamic_adar",
        "aa",
        "effective_resistance",
        "effective-resistance",
        "er",
        "approx_effective_resistance",
        "approx_er",
        "random",
        "rand",
        "degree",
        "feature_cosine",
        "feature-cosine",
    }

    _DISTANCE_METRICS = {"effective_resistance", "approx_effective_resistance"}

    def __init__(self, data: Data, device: str, tie_break: str | None = None,
                 gpu: int | None = None) -> None:
        self.data = data
        self.device = device
        self.num_nodes = data.num_nodes
        self.num_edges = data.edge_index.size(1)
        self.verbose: bool = False
        self.tie_break = tie_break or os.environ.get("GSPARSE_TIE_BREAK", "numpy")
        if self.tie_break not in ("numpy", "stable"):
            raise ValueError(f"tie_break must be 'numpy' or 'stable', got {self.tie_break!r}")
        if gpu is None:
            gpu = _device_index(device)
        self._ctx = Context(gpu)
        ei = data.edge_index
        if ei.is_cuda and ei.device.index == self._ctx.device:
            src = ei[0].contiguous().to(torch.int64)
            dst = ei[1].contiguous().to(torch.int64)
        else:
            e = ei.detach().cpu().numpy().astype(np.int64, copy=False)
            src = np.ascontiguousarray(e[0])
            dst = np.ascontiguousarray(e[1])
        self._ctx.set_graph_edge_index(int(self.num_nodes), src, dst)
        self._engine = Engine(self._ctx)
        self._adj = None
        self._score_cache: Dict[str, np.ndarray] = {}
        self.last_selection: dict = {}

    # ------------------------------------------------------------------ adj
    @property
    def adj(self) -> sp.csr_matrix:
        """Canonical CSR (core.py:71-74), downloaded from the device on first use."""
        if self._adj is None:
            indptr, indices, data = self._ctx.csr()
            a = sp.csr_matrix((data, indices, indptr), shape=(self.num_nodes, self.num_nodes))
            a.has_sorted_indices = True
            self._adj = a
        return self._adj

    @adj.setter
    def adj(self, value):
        self._adj = value

    # ------------------------------------------------------------- helpers
    def _scores_to_cost(self, scores: np.ndarray, metric: str) -> np.ndarray:
        """Proximity -> distance transform of Simas et al. (core.py:82-116)."""
        metric_key = self._normalize_metric_name(metric)
        if metric_key in self._DISTANCE_METRICS:
            safe = np.maximum(scores, 1e-10)
            similarity = 1.0 / safe
        else:
            similarity = scores.copy()
        s_max = similarity.max()
        if s_max <= 0:
            return np.ones_like(scores)
        proximity = similarity / s_max
        nonzero = proximity[proximity > 0]
        floor = (nonzero.min() * 0.01) if len(nonzero) > 0 else 1e-6
        proximity[proximity <= 0] = floor
        return 1.0 / proximity - 1.0

    def _normalize_metric_name(self, metric: str) -> str:
        """core.py:118-138."""
        metric_lower = metric.lower().replace("-", "_").replace(" ", "_")
        if metric_lower in {"jaccard"}:
            return "jaccard"
        if metric_lower in {"adamic_adar", "aa"}:
            return "adamic_adar"
        if metric_lower in {"effective_resistance", "er"}:
            return "effective_resistance"
        if metric_lower in {"approx_effective_resistance", "approx_er"}:
            return "approx_effective_resistance"
        if metric_lower in {"random", "rand"}:
            return "random"
        if metric_lower in {"degree"}:
            return "degree"
        if metric_lower in {"feature_cosine"}:
            return "feature_cosine"
        raise ValueError(
            f"Metric '{metric}' not supported. " f"Choose from: {self.SUPPORTED_METRICS}"
        )

    # --------------------------------------------------------------- scores
    def compute_scores(self, metric: str) -> np.ndarray:
        """Compute or retrieve cached edge scores (core.py:140-191), CSR order."""
        metric_key = self._normalize_metric_name(metric)
        if metric_key in self._score_cache:
            return self._score_cache[metric_key]
        eng = self._engine
        if metric_key == "jaccard":
            scores = eng.jaccard()
        elif metric_key == "adamic_adar":
            scores = eng.adamic_adar()
        elif metric_key == "effective_resistance":
            scores = eng.exact_er()
        elif metric_key == "approx_effective_resistance":
            scores = eng.approx_er()
        elif metric_key == "random":
            # legacy global NumPy RNG, exactly as core.py:166
            scores = np.random.rand(eng.nnz)
        elif metric_key == "degree":
            scores = eng.degree()
        elif metric_key == "feature_cosine":
            x = self.data.x if getattr(self.data, "x", None) is not None else None
            if x is None:
                raise ValueError("feature_cosine requires node features (data.x)")
            if x.is_cuda and x.device.index == self._ctx.device:
                scores = eng.feature_cosine(x)
            else:
                scores = eng.feature_cosine(x.detach().cpu().numpy())
        else:  # pragma: no cover - unreachable, mirrors core.py:186-188
            raise ValueError(f"Internal error: Unhandled metric '{metric_key}'")
        self._score_cache[metric_key] = scores
        return scores

    # ------------------------------------------------------------ selection
    def _select_mask(self, scores: np.ndarray, num_keep: int, keep_lowest: bool) -> np.ndarray:
        mask, cut, beyond, tied = self._engine.topk_mask(scores, self.num_edges, num_keep,
                                                         keep_lowest)
        need = num_keep - beyond
        ambiguous = 0 < need < tied
        self.last_selection = {"cut": cut, "beyond": beyond, "tied": tied, "need": need,
                               "ambiguous": ambiguous}
        if ambiguous and self.tie_break == "numpy":
            # The reference's unstable np.argsort orders the tie block; reproduce
            # it by making that same call (core.py:233-240).
            mask = numpy_topk_mask(scores, self.num_edges, num_keep, keep_lowest)
        return mask

    def sparsify(self, metric: str, retention_ratio: float, return_mask: bool = False,
                 keep_lowest: bool = False):
        """Keep exactly the top (bottom) ``int(E*r)`` edges by score (core.py:193-249)."""
        if not 0 < retention_ratio <= 1:
            raise ValueError(f"retention_ratio must be in (0, 1], got {retention_ratio}")
        if retention_ratio == 1.0:
            if return_mask:
                return self.data.clone(), torch.ones(self.num_edges, dtype=torch.bool)
            return self.data.clone()
        scores = self.compute_scores(metric)
        num_keep = int(self.num_edges * retention_ratio)
        mask = self._select_mask(scores, num_keep, keep_lowest)
        sparse_edge_index = self.data.edge_index[:, torch.from_numpy(mask).to(
            self.data.edge_index.device)].to(self.device)
        sparse_data = self.data.clone()
        sparse_data.edge_index = sparse_edge_index
        if return_mask:
            return sparse_data, torch.from_numpy(mask)
        return sparse_data

    def sparsify_metric_backbone(self, metric: str, epsilon: float = 1e-9):
        """Global metric backbone with costs from ``_scores_to_cost`` (core.py:251-279)."""
        distances = self._scores_to_cost(self.compute_scores(metric), metric)
        sparse_data, stats = compute_metric_backbone(
            self.data, distances, epsilon=epsilon, verbose=self.verbose, _ctx=self._ctx
        )
        return sparse_data.to(self.device), stats

    def sparsify_sampled(self, metric: str, retention_ratio: float, seed: int = 42,
                         return_mask: bool = False):
        """Score-proportional sampling without replacement (core.py:281-357).

        NumPy's ``Generator.choice`` stream defines the result; it runs on the
        host exactly as in the reference."""
        if not 0 < retention_ratio <= 1:
            raise ValueError(f"retention_ratio must be in (0, 1], got {retention_ratio}")
        if retention_ratio == 1.0:
            if return_mask:
                return self.data.clone(), torch.ones(self.num_edges, dtype=torch.bool)
            return self.data.clone()
        scores = self.compute_scores(metric)
        mask = sampled_mask(scores, self.num_edges, retention_ratio, seed)
        sparse_edge_index = self.data.edge_index[:, torch.from_numpy(mask).to(
            self.data.edge_index.device)].to(self.device)
        sparse_data = self.data.clone()
        sparse_data.edge_index = sparse_edge_index
        if return_mask:
            return sparse_data, torch.from_numpy(mask)
        return sparse_data

    def sparsify_degree_aware(self, metric: str, retention_ratio: float,
                              min_edges_per_node: int = 1, return_mask: bool = False):
        """Per-node minimum budget, then global fill (core.py:359-461).

        Same result as the reference's O(N*E) loops: each node's guaranteed
        columns are chosen by the same ``np.argsort`` over its incident scores,
        and the fill takes the first non-guaranteed entries of
        ``np.argsort(scores)[::-1]`` -- both on the device, with the reference's
        own calls only where its argsort order decides."""
        if not 0 < retention_ratio <= 1:
            raise ValueError(f"retention_ratio must be in (0, 1], got {retention_ratio}")
        if retention_ratio == 1.0:
            if return_mask:
                return self.data.clone(), torch.ones(self.num_edges, dtype=torch.bool)
            return self.data.clone()
        scores = self.compute_scores(metric)
        mask = degree_aware_mask_device(self._engine, scores, self.data.edge_index.cpu().numpy(),
                                        self.num_nodes, self.num_edges, retention_ratio,
                                        min_edges_per_node)
        sparse_edge_index = self.data.edge_index[:, torch.from_numpy(mask).to(
            self.data.edge_index.device)].to(self.device)
        sparse_data = self.data.clone()
        sparse_data.edge_index = sparse_edge_index
        if return_mask:
            return sparse_data, torch.from_numpy(mask)
        return sparse_data

    def get_retention_curve_data(self, metric: str, retention_rates: list[float]) -> list[Data]:
        """core.py:463-480."""
        return [self.sparsify(metric, rate) for rate in retention_rates]

    @property
    def stats(self) -> dict:
        """core.py:482-490."""
        return {
            "num_nodes": self.num_nodes,
            "num_edges": self.num_edges,
            "density": self.num_edges / (self.num_nodes * (self.num_nodes - 1)),
            "avg_degree": self.num_edges / self.num_nodes,
        }


SparsificationEngine = GraphSparsifier
