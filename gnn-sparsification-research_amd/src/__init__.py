"""Drop-in ``src`` namespace: the reference's sparsification entry points,
backed by gsparse (MI355X).  Only the hot-path package is provided; the
reference's models / training modules are out of scope; ``src.data`` is a
local-file / synthetic loader (the reference's own module is absent)."""

from .data import SAFE_DATASETS, DatasetLoader  # noqa: F401
from .sparsification import GraphSparsifier  # noqa: F401
