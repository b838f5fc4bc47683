"""``src.sparsification`` drop-in (reference: src/sparsification/__init__.py)."""

from gsparse import (  # noqa: F401
    GraphSparsifier,
    calculate_adamic_adar_scores,
    calculate_approx_effective_resistance_scores,
    calculate_effective_resistance_scores,
    calculate_feature_cosine_scores,
    calculate_jaccard_scores,
    compute_geodesic_preservation,
    compute_topology_metrics,
    compute_topology_preservation,
    precompute_random_scores,
    random_sparsify,
)

__all__ = [
    "GraphSparsifier",
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
