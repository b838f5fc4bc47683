"""Dataset loader -- stands in for the reference's ``src/data`` (``DatasetLoader``,
``SAFE_DATASETS``), which its repository does not contain (``.gitignore`` swallowed
it).  Only the call-site contract is known and kept:

    loader = DatasetLoader(root=...)                       # roman_empire_gpu.py:437
    data, num_features, num_classes = loader.get_dataset(  # run_ablation.py:99,
        name, device, split_idx=None)                      # run_real_transfer.py:123

There is no network: nothing is downloaded.  A dataset is read from local
files under ``root`` in one of these layouts (first match wins):

* ``{root}/{name}.npz`` -- ``edge_index`` [2, E] (or ``edges`` [E, 2]), optional
  ``x`` [n, f], ``y`` [n], ``num_nodes``, and ``train_mask`` / ``val_mask`` /
  ``test_mask`` ([n] or [n, S] for S splits);
* the same file, or ``{root}/{name}/raw/{name}.npz``, in the layout of the
  heterophilous benchmark files (Platonov et al.; roman_empire,
  amazon_ratings, minesweeper, tolokers, questions): ``node_features``,
  ``node_labels``, ``edges`` [E, 2], ``train_masks`` / ``val_masks`` /
  ``test_masks`` [S, n];
* ``synthetic-<config>`` names need no file: the SURVEY §8(d) stand-ins
  (``synthetic-cora``, ``synthetic-roman_empire``, ``synthetic-ogbn_arxiv``,
  ``synthetic-rmat<scale>``), with seeded random labels and a 60/20/20 split.

Every edge list is made canonical on the device (``gs_coalesce_edges``): both
directions, duplicates removed, sorted by (row, col) -- what PyG's
``to_undirected`` does to these datasets -- so CSR-ordered scores and
``edge_index``-ordered masks line up (SURVEY §0 finding 4).  ``split_idx``
picks one column of [n, S] masks (WebKB / Actor / heterophilous: 10 splits).
"""

from __future__ import annotations

import ctypes
import os
from typing import Tuple

import numpy as np
import torch

from ._lib import GS_HOST, Context, ptr
from .data import Data

# the dataset names the reference's callers pass (run_ablation.py:46-47,361;
# run_real_transfer.py:65-70; run_hpo_robustness.py:80; roman_empire_gpu.py:76)
SAFE_DATASETS = [
    "cora", "citeseer", "pubmed", "actor", "cornell", "texas", "wisconsin",
    "roman_empire", "polblogs", "flickr", "physics", "cs", "corafull", "ppi",
]

_HETERO_KEYS = ("node_features", "node_labels", "edges")
_SYNTHETIC = {
    # name: (graph builder, n, feature dim, feature kind, classes)
    "cora": ("chung_lu", 2_708, 1_433, "bow", 7),
    "roman_empire": ("roman_like", 22_662, 300, "normal", 18),
    "ogbn_arxiv": ("citation_like", 169_343, 128, "normal", 40),
}

_CTX = None


def _context(ctx: Context | None) -> Context:
    global _CTX
    if ctx is not None:
        return ctx
    if _CTX is None:
        _CTX = Context()
    return _CTX


def coalesce_edges(edge_index, num_nodes: int, undirected: bool = True,
                   remove_self_loops: bool = False, ctx: Context | None = None) -> np.ndarray:
    """Canonical int64 [2, m] edge list (gs_coalesce_edges): with ``undirected``
    every reversed pair is added; sorted by (row, col), duplicates removed."""
    ei = np.asarray(edge_index, dtype=np.int64).reshape(2, -1)
    E = int(ei.shape[1])
    src = np.ascontiguousarray(ei[0])
    dst = np.ascontiguousarray(ei[1])
    cap = max(2 * E if undirected else E, 1)
    out_s = np.empty(cap, dtype=np.int64)
    out_d = np.empty(cap, dtype=np.int64)
    m = ctypes.c_int64(cap)
    _context(ctx).call("gs_coalesce_edges", int(num_nodes), E, ptr(src), ptr(dst),
                       int(bool(undirected)), int(bool(remove_self_loops)), ptr(out_s), ptr(out_d),
                       ctypes.byref(m), GS_HOST)
    return np.stack([out_s[: m.value], out_d[: m.value]])


def _pick_split(mask, split_idx):
    m = np.asarray(mask).astype(bool)
    if m.ndim == 2 and split_idx is not None:
        if not 0 <= split_idx < m.shape[1]:
            raise ValueError(f"split_idx {split_idx} out of range: {m.shape[1]} splits")
        m = m[:, split_idx]
    return torch.from_numpy(np.ascontiguousarray(m))


def _random_split(n: int, seed: int):
    rng = np.random.default_rng(seed)
    perm = rng.permutation(n)
    a, b = int(0.6 * n), int(0.8 * n)
    masks = []
    for lo, hi in ((0, a), (a, b), (b, n)):
        m = np.zeros(n, dtype=bool)
        m[perm[lo:hi]] = True
        masks.append(m)
    return masks


class DatasetLoader:
    """Local-file / synthetic dataset loader (see the module docstring)."""

    def __init__(self, root: str = "data", ctx: Context | None = None):
        self.root = str(root)
        self._ctx = ctx

    def _find(self, key: str):
        for p in (os.path.join(self.root, f"{key}.npz"),
                  os.path.join(self.root, key, "raw", f"{key}.npz"),
                  os.path.join(self.root, key, f"{key}.npz")):
            if os.path.isfile(p):
                return p
        return None

    def get_dataset(self, name: str, device="cpu",
                    split_idx: int | None = None) -> Tuple[Data, int, int]:
        """-> (Data(x, edge_index, y, train/val/test_mask), num_features, num_classes)."""
        key = name.lower().replace("-", "_")
        if key.startswith("synthetic_"):
            data = self._synthetic(key[len("synthetic_"):], split_idx)
        else:
            path = self._find(key)
            if path is None:
                raise FileNotFoundError(
                    f"dataset {name!r}: no local file under {self.root!r} (looked for {key}.npz, "
                    f"{key}/raw/{key}.npz); nothing is downloaded -- place the file there or use "
                    f"a 'synthetic-*' stand-in")
            data = self._from_npz(path, split_idx)
        nf = 0 if data.x is None else int(data.x.shape[1])
        y = getattr(data, "y", None)
        nc = 0 if y is None or y.numel() == 0 else int(y.max().item()) + 1
        return data.to(device), nf, nc

    def _from_npz(self, path: str, split_idx):
        with np.load(path, allow_pickle=False) as z:
            keys = set(z.files)
            if all(k in keys for k in _HETERO_KEYS):
                x = z["node_features"]
                y = z["node_labels"]
                edges = np.asarray(z["edges"], dtype=np.int64).T
                masks = [z[k].T if k in keys else None
                         for k in ("train_masks", "val_masks", "test_masks")]
                n = int(x.shape[0])
            else:
                if "edge_index" in keys:
                    edges = np.asarray(z["edge_index"], dtype=np.int64)
                elif "edges" in keys:
                    edges = np.asarray(z["edges"], dtype=np.int64).T
                else:
                    raise ValueError(f"{path}: neither edge_index nor edges")
                x = z["x"] if "x" in keys else None
                y = z["y"] if "y" in keys else None
                if "num_nodes" in keys:
                    n = int(z["num_nodes"])
                elif x is not None:
                    n = int(x.shape[0])
                else:
                    n = int(edges.max()) + 1 if edges.size else 0
                masks = [z[k] if k in keys else None for k in ("train_mask", "val_mask", "test_mask")]
        ei = coalesce_edges(edges, n, undirected=True, ctx=self._ctx)
        data = Data(x=None if x is None else torch.from_numpy(np.ascontiguousarray(x)),
                    edge_index=torch.from_numpy(ei), num_nodes=n)
        if y is not None:
            data.y = torch.from_numpy(np.ascontiguousarray(y).astype(np.int64))
        for k, m in zip(("train_mask", "val_mask", "test_mask"), masks):
            if m is not None:
                setattr(data, k, _pick_split(m, split_idx))
        return data

    def _synthetic(self, key: str, split_idx):
        from . import graphs

        if key.startswith("rmat"):
            scale = int(key[4:] or 18)
            n = 1 << scale
            ei = graphs.rmat(scale, 8, seed=0)
            f, kind, ncls = 0, None, 0
        elif key in _SYNTHETIC:
            builder, n, f, kind, ncls = _SYNTHETIC[key]
            ei = getattr(graphs, builder)()
        else:
            raise ValueError(f"unknown synthetic dataset {key!r}: "
                             f"{sorted(_SYNTHETIC) + ['rmat<scale>']}")
        ei = coalesce_edges(ei, n, undirected=True, ctx=self._ctx)
        x = torch.from_numpy(graphs.features(n, f, seed=1, kind=kind)) if f else None
        data = Data(x=x, edge_index=torch.from_numpy(ei), num_nodes=n)
        if ncls:
            rng = np.random.default_rng(2)
            data.y = torch.from_numpy(rng.integers(0, ncls, size=n).astype(np.int64))
            seed = 3 + (split_idx or 0)
            for k, m in zip(("train_mask", "val_mask", "test_mask"), _random_split(n, seed)):
                setattr(data, k, torch.from_numpy(m))
        return data
