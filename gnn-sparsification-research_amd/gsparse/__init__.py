"""gsparse -- MI355X-native graph-sparsification edge scoring.

Drop-in for the reference's ``src/sparsification`` package: the same public
names, backed by libgsparse.so (hand-written HIP for gfx950).  Importing the
package does not touch the GPU; the first scorer call does, and fails loudly
(``GsparseUnavailable``) when the HIP library or device is missing.
"""

from ._lib import GsparseError, GsparseUnavailable
from .core import GraphSparsifier, SparsificationEngine
from .data import Data
from .metric_backbone import compute_metric_backbone
from .metrics import (
    calculate_adamic_adar_scores,
    calculate_approx_effective_resistance_scores,
    calculate_effective_resistance_scores,
    calculate_feature_cosine_scores,
    calculate_jaccard_scores,
    compute_geodesic_preservation,
    compute_topology_metrics,
    compute_topology_preservation,
)
from .random import precompute_random_scores, random_sparsify

__all__ = [
    "GraphSparsifier",
    "SparsificationEngine",
    "Data",
    "GsparseError",
    "GsparseUnavailable",
    "compute_metric_backbone",
    "calculate_jaccard_scores",
    "calculate_adamic_adar_scores",
    "calculate_effective_resistance_scores",
    "calculate_approx_effective_resistance_scores",
    "calculate_feature_cosine_scores",
    "compute_geodesic_preservation",
    "compute_topology_metrics",
    "compute_topology_preservation",
    "precompute_random_scores",
    "random_sparsify",
]
