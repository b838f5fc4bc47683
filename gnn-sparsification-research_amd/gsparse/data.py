"""Graph container: ``torch_geometric.data.Data`` when PyG is installed,
otherwise a minimal stand-in with the attributes the reference path touches
(``edge_index``, ``x``, ``num_nodes``, ``clone()``, ``to()``, extra keys)."""

from __future__ import annotations

try:  # pragma: no cover - PyG is not installed in this image
    from torch_geometric.data import Data  # type: ignore
except Exception:  # noqa: BLE001
    import torch

    class Data:  # type: ignore[no-redef]
        def __init__(self, x=None, edge_index=None, num_nodes=None, **kwargs):
            self.x = x
            self.edge_index = edge_index
            self._num_nodes = num_nodes
            for k, v in kwargs.items():
                setattr(self, k, v)

        @property
        def num_nodes(self):
            if self._num_nodes is not None:
                return int(self._num_nodes)
            if self.x is not None:
                return int(self.x.shape[0])
            if self.edge_index is not None and self.edge_index.numel() > 0:
                return int(self.edge_index.max()) + 1
            return 0

        @num_nodes.setter
        def num_nodes(self, v):
            self._num_nodes = v

        @property
        def num_edges(self):
            return 0 if self.edge_index is None else int(self.edge_index.size(1))

        def keys(self):
            return [k for k in self.__dict__ if not k.startswith("_") and k != "_num_nodes"]

        def _apply(self, fn):
            out = Data.__new__(Data)
            for k, v in self.__dict__.items():
                out.__dict__[k] = fn(v) if isinstance(v, torch.Tensor) else v
            return out

        def clone(self):
            return self._apply(lambda t: t.clone())

        def to(self, device, *args, **kwargs):
            return self._apply(lambda t: t.to(device, *args, **kwargs))

        def cpu(self):
            return self.to("cpu")

        def __repr__(self):
            parts = []
            for k, v in self.__dict__.items():
                if k == "_num_nodes":
                    continue
                if isinstance(v, torch.Tensor):
                    parts.append(f"{k}={list(v.shape)}")
                elif v is not None:
                    parts.append(f"{k}={v}")
            return f"Data({', '.join(parts)})"
