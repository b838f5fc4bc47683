"""ctypes binding of libgsparse.so (include/gsparse.h).

The product path has NO CPU fallback: if the HIP library or a gfx950 GPU is
missing, :func:`lib` / :class:`Context` raise ``GsparseUnavailable``.
"""

from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GSPARSE_LIB", os.path.join(_HERE, "libgsparse.so"))

GS_HOST, GS_DEVICE = 0, 1
GS_OK, GS_EINVAL, GS_EHIP, GS_ENOMEM, GS_ESTATE, GS_EUNSUPPORTED, GS_EINDEX = 0, -1, -2, -3, -4, -5, -6

_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_u64 = ctypes.c_uint64
_f64 = ctypes.c_double
_vp = ctypes.c_void_p
_int = ctypes.c_int

# name -> (restype, argtypes); mirrors include/gsparse.h one to one.
SIGNATURES = {
    "gs_api_version": (_int, []),
    "gs_last_error": (ctypes.c_char_p, []),
    "gs_device_count": (_int, [ctypes.POINTER(_int)]),
    "gs_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "gs_destroy": (None, [_vp]),
    "gs_set_stream": (_int, [_vp, _vp]),
    "gs_stream_wait": (_int, [_vp, _vp]),
    "gs_stream_signal": (_int, [_vp, _vp]),
    "gs_synchronize": (_int, [_vp]),
    "gs_set_async": (_int, [_vp, _int]),
    "gs_profile_enable": (_int, [_vp, _int]),
    "gs_profile_reset": (_int, [_vp]),
    "gs_profile_get": (_int, [_vp, _int, ctypes.c_char_p, _int, ctypes.POINTER(_i64),
                              ctypes.POINTER(_f64), ctypes.POINTER(_f64)]),
    "gs_graph_from_edge_index": (_int, [_vp, _i64, _i64, _vp, _vp, _int]),
    "gs_coalesce_edges": (_int, [_vp, _i64, _i64, _vp, _vp, _int, _int, _vp, _vp, _vp, _int]),
    "gs_graph_from_csr": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _int]),
    "gs_graph_shape": (_int, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i64), ctypes.POINTER(_int)]),
    "gs_graph_copy_csr": (_int, [_vp, _vp, _vp, _vp, _int]),
    "gs_jaccard": (_int, [_vp, _i64, _i64, _vp, _int]),
    "gs_jaccard_part": (_int, [_vp, _int, _int, _vp, _int]),
    "gs_jaccard_shares": (_int, [_vp, _int, _vp, _vp]),
    "gs_jaccard_part_counts": (_int, [_vp, _int, _int, _vp, _int]),
    "gs_jaccard_from_counts": (_int, [_vp, _int, _vp, _i64, _int, _vp, _int]),
    "gs_adamic_adar": (_int, [_vp, _vp, _int, _i64, _i64, _vp, _int]),
    "gs_degree": (_int, [_vp, _i64, _i64, _vp, _int]),
    "gs_feature_cosine_f32": (_int, [_vp, _vp, _i64, _int, _i64, _i64, _vp, _int]),
    "gs_feature_cosine_f64": (_int, [_vp, _vp, _i64, _int, _i64, _i64, _vp, _int]),
    "gs_er_prepare": (_int, [_vp, _i64, _f64, ctypes.POINTER(_i64)]),
    "gs_er_project_rows": (_int, [_vp, _i64, _i64, _vp, _int, _f64]),
    "gs_er_project_pcg64": (_int, [_vp, _u64, _u64, _u64, _u64, _f64]),
    "gs_er_project_pcg64_cols": (_int, [_vp, _u64, _u64, _u64, _u64, _f64, _i64, _i64]),
    "gs_er_project_rows_cols": (_int, [_vp, _i64, _i64, _vp, _int, _f64, _i64, _i64]),
    "gs_er_solve": (_int, [_vp, _i64, _i64, _i32, _f64, _i32]),
    "gs_er_scores": (_int, [_vp, _i64, _i64, _i64, _i64, _int, _vp, _int]),
    "gs_er_iterations": (_int, [_vp, _vp, _int]),
    "gs_er_copy_z": (_int, [_vp, _i64, _i64, _vp, _int]),
    "gs_er_split": (_int, [_i64, _i32, _vp]),
    "gs_topk_mask": (_int, [_vp, _vp, _int, _i64, _i64, _i64, _int, _vp, _int,
                            ctypes.POINTER(_f64), ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "gs_segment_argmax": (_int, [_vp, _vp, _int, _i64, _vp, _int, _i64, _i64, _vp, _int]),
    "gs_metric_backbone": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _int, _f64, _vp, _int,
                                  ctypes.POINTER(_i64)]),
    "gs_metric_backbone_part": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _int, _f64, _int,
                                       _int, _vp, _int, ctypes.POINTER(_i64)]),
    "gs_bb_begin": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _int, _f64, _int, _int,
                           ctypes.POINTER(_i32)]),
    "gs_bb_landmarks_io": (_int, [_vp, _vp, _vp, _int, _int]),
    "gs_bb_certify": (_int, [_vp, _int, _int]),
    "gs_bb_state_io": (_int, [_vp, _vp, _int, _int]),
    "gs_bb_plan": (_int, [_vp, ctypes.POINTER(_i64)]),
    "gs_bb_search": (_int, [_vp, _i64, _i64, _int, _int]),
    "gs_bb_finish": (_int, [_vp, _vp, _int, ctypes.POINTER(_i64)]),
    "gs_bb_classes": (_int, [_vp, _int]),
    "gs_jsel_begin": (_int, [_vp, _int, _int, _vp, _int, _i64, _int, _vp, _vp, _int]),
    "gs_jsel_step": (_int, [_vp, _vp, ctypes.POINTER(_int)]),
    "gs_jsel_result": (_int, [_vp, ctypes.POINTER(_f64), ctypes.POINTER(_i64), ctypes.POINTER(_i64),
                              ctypes.POINTER(_i64)]),
    "gs_jsel_tie_positions": (_int, [_vp, _vp, _i64, _int]),
    "gs_jsel_keep": (_int, [_vp, _vp, _i64, _int, _i64, _vp, _int]),
    "gs_jsel_mask": (_int, [_vp, _int, _vp, _i64, _int, _vp, _int]),
    "gs_bb_class_counts": (_int, [_vp, _vp, _int, _vp, _i64, _int, ctypes.POINTER(_i64)]),
    "gs_exact_er": (_int, [_vp, _vp, _int, ctypes.POINTER(_i32)]),
    "gs_pair_distances": (_int, [_vp, _i64, _i64, _vp, _vp, _vp, _i64, _int, _i64, _vp, _vp,
                                 _vp]),
    "gs_common_neighbors": (_int, [_vp, _vp, _int]),
    "gs_clustering": (_int, [_vp, ctypes.POINTER(_f64), _vp, _int]),
    "gs_components": (_int, [_vp, _vp, _int, ctypes.POINTER(_i64), ctypes.POINTER(_i64)]),
    "gs_fiedler": (_int, [_vp, _f64, _i32, ctypes.POINTER(_f64), ctypes.POINTER(_i32)]),
}


# entry points that touch no caller buffers on the device: no stream ordering
_NO_ORDER = frozenset({"gs_set_stream", "gs_stream_wait", "gs_stream_signal", "gs_set_async",
                       "gs_profile_enable", "gs_profile_reset", "gs_profile_get",
                       "gs_graph_shape", "gs_synchronize"})


class GsparseUnavailable(RuntimeError):
    """libgsparse.so (HIP, gfx950) or a usable MI355X device is missing."""


class GsparseError(RuntimeError):
    pass


_LIB = None
_LOCK = threading.Lock()


def lib(path: str | None = None):
    """Load libgsparse.so and bind every entry point of include/gsparse.h."""
    global _LIB
    with _LOCK:
        if _LIB is not None and path is None:
            return _LIB
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise GsparseUnavailable(
                f"{p} not found: build it with `make -C gnn-sparsification-research_amd/csrc` "
                "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if path is None:
            _LIB = L
        return L


def check(rc: int, what: str = ""):
    if rc == GS_OK:
        return
    msg = lib().gs_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == GS_EINVAL:
        raise ValueError(text)
    if rc == GS_EUNSUPPORTED:
        raise NotImplementedError(text)
    if rc == GS_EINDEX:
        raise IndexError(text)
    if rc == GS_ENOMEM:
        raise MemoryError(text)
    raise GsparseError(f"[{rc}] {text}")


def ptr(a) -> int:
    """Data pointer of a contiguous numpy array or torch tensor."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return a.data_ptr()


def device_count() -> int:
    n = _int(0)
    rc = lib().gs_device_count(ctypes.byref(n))
    if rc != GS_OK:
        return 0
    return n.value


def _torch_current_device() -> int | None:
    """torch's current CUDA device when torch has initialised CUDA in this
    process (a caller's ``torch.cuda.set_device(k)`` -- roman_empire_gpu.py:209
    before ``GraphSparsifier(full_graph, device='cpu')`` at :213), else None.
    Never initialises CUDA itself."""
    import sys

    torch = sys.modules.get("torch")
    if torch is None:
        return None
    try:
        if not torch.cuda.is_initialized():
            return None
        return int(torch.cuda.current_device())
    except Exception:
        return None


def default_device() -> int:
    """Device of a context created without an explicit ordinal:
    $GSPARSE_DEVICE, else torch's current device once torch has initialised
    CUDA (the caller's set_device), else $LOCAL_RANK (modulo the visible GPUs),
    else 0."""
    env = os.environ.get("GSPARSE_DEVICE")
    if env is not None:
        return int(env)
    cur = _torch_current_device()
    if cur is not None:
        return cur
    lr = os.environ.get("LOCAL_RANK")
    if lr is not None:
        # one process per GPU (roman_empire_gpu.py:347); more ranks than visible
        # GPUs (a rehearsal on a smaller box) share them round-robin
        cnt = device_count()
        return int(lr) % cnt if cnt > 0 else int(lr)
    return 0


class Context:
    """One libgsparse context: a HIP stream, device buffers, one resident graph."""

    def __init__(self, device: int | None = None):
        L = lib()
        self.device = default_device() if device is None else int(device)
        h = _vp()
        rc = L.gs_create(self.device, ctypes.byref(h))
        if rc != GS_OK:
            msg = L.gs_last_error().decode(errors="replace")
            raise GsparseUnavailable(f"gs_create(device={self.device}) failed: {msg}")
        self._h = h
        self._L = L
        self._async = False

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            self._L.gs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _torch_stream(self):
        """torch's current stream on this device, or None when torch has not
        touched the GPU in this process (then no torch work can be pending)."""
        try:
            import torch
        except ImportError:  # pragma: no cover - torch is a dependency
            return None
        if not torch.cuda.is_initialized():
            return None
        return torch.cuda.current_stream(self.device).cuda_stream

    def call(self, name: str, *args):
        """Call a libgsparse entry point on this context.

        Compute calls are ordered after torch's current stream first: device
        buffers handed in (inputs torch just produced, or caching-allocator
        blocks torch's stream last used) are ready before the library's own
        stream touches them.  In async mode torch's stream is then ordered
        after the library's, so device outputs are complete for torch too."""
        ts = None if name in _NO_ORDER else self._torch_stream()
        if ts is not None:
            check(self._L.gs_stream_wait(self._h, ts), "gs_stream_wait")
        check(getattr(self._L, name)(self._h, *args), name)
        if ts is not None and self._async:
            check(self._L.gs_stream_signal(self._h, ts), "gs_stream_signal")

    def set_async(self, on: bool):
        self.call("gs_set_async", int(on))
        self._async = bool(on)

    # ---- profiling -------------------------------------------------------
    def profile(self, on: bool = True):
        self.call("gs_profile_enable", int(on))

    def profile_reset(self):
        self.call("gs_profile_reset")

    def profile_read(self) -> dict:
        out = {}
        i = 0
        buf = ctypes.create_string_buffer(128)
        while True:
            lc, ms, by = _i64(0), _f64(0), _f64(0)
            rc = self._L.gs_profile_get(self._h, i, buf, 128, ctypes.byref(lc), ctypes.byref(ms),
                                        ctypes.byref(by))
            if rc != GS_OK:
                break
            out[buf.value.decode()] = {"launches": lc.value, "ms": ms.value, "bytes": by.value}
            i += 1
        return out

    def synchronize(self):
        self.call("gs_synchronize")

    def set_stream(self, stream_ptr: int | None):
        self.call("gs_set_stream", stream_ptr)

    # ---- graph -----------------------------------------------------------
    def set_graph_edge_index(self, n: int, src, dst):
        """src/dst: int64 numpy arrays (host) or torch int64 CUDA tensors."""
        loc = GS_HOST if isinstance(src, np.ndarray) else GS_DEVICE
        E = int(src.shape[0])
        self.call("gs_graph_from_edge_index", n, E, ptr(src), ptr(dst), loc)

    def set_graph_csr(self, n: int, indptr: np.ndarray, indices: np.ndarray,
                      data: np.ndarray | None):
        indptr = np.ascontiguousarray(indptr, dtype=np.int64)
        indices = np.ascontiguousarray(indices, dtype=np.int32)
        if data is not None:
            data = np.ascontiguousarray(data, dtype=np.float64)
        self._keep = (indptr, indices, data)
        self.call("gs_graph_from_csr", n, int(indices.shape[0]), ptr(indptr), ptr(indices),
                  ptr(data), GS_HOST)

    def shape(self):
        n, nnz, sym = _i64(0), _i64(0), _int(0)
        self.call("gs_graph_shape", ctypes.byref(n), ctypes.byref(nnz), ctypes.byref(sym))
        return n.value, nnz.value, bool(sym.value)

    def csr(self):
        n, nnz, _ = self.shape()
        indptr = np.empty(n + 1, dtype=np.int64)
        indices = np.empty(nnz, dtype=np.int32)
        data = np.empty(nnz, dtype=np.float64)
        self.call("gs_graph_copy_csr", ptr(indptr), ptr(indices), ptr(data), GS_HOST)
        return indptr, indices, data
