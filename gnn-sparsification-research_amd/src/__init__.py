"""Drop-in ``src`` namespace: the reference's sparsification entry points,
backed by gsparse (MI355X).  Only the hot-path package is provided; the
reference's models / training / data modules are out of scope."""

from .sparsification import GraphSparsifier  # noqa: F401
