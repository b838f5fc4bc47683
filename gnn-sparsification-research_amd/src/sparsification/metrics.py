"""``src.sparsification.metrics`` drop-in (reference metrics.py)."""

from gsparse.metrics import (  # noqa: F401
    calculate_adamic_adar_scores,
    calculate_approx_effective_resistance_scores,
    calculate_effective_resistance_scores,
    calculate_feature_cosine_scores,
    calculate_jaccard_scores,
    compute_geodesic_preservation,
    compute_topology_metrics,
    compute_topology_preservation,
)
