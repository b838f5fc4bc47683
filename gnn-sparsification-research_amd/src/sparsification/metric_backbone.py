"""``src.sparsification.metric_backbone`` drop-in (reference metric_backbone.py)."""

from gsparse.metric_backbone import compute_metric_backbone, verify_geodesic_preservation  # noqa: F401
