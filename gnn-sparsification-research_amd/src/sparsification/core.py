"""``src.sparsification.core`` drop-in (reference core.py:24)."""

from gsparse.core import GraphSparsifier, SparsificationEngine  # noqa: F401
