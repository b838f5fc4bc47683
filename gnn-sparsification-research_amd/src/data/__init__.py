"""Drop-in ``src.data``: ``DatasetLoader`` / ``SAFE_DATASETS`` (src/__init__.py:33,
run_ablation.py:34) from gsparse's local-file / synthetic loader."""

from gsparse.loader import SAFE_DATASETS, DatasetLoader  # noqa: F401
