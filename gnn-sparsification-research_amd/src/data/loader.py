"""Drop-in ``src.data.loader`` (run_real_transfer.py:43)."""

from gsparse.loader import SAFE_DATASETS, DatasetLoader, coalesce_edges  # noqa: F401
