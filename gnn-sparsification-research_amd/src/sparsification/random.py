"""``src.sparsification.random`` drop-in (reference random.py)."""

from gsparse.random import precompute_random_scores, random_sparsify  # noqa: F401
