"""Scorer orchestration over one libgsparse context (host side of the hot path).

Everything numeric runs in libgsparse.so (HIP, gfx950).  The host keeps only
what the reference defines through NumPy itself and that must therefore be
evaluated by NumPy to stay bit-identical: the per-node Adamic-Adar weights
c = 1/sqrt(max(log(deg+1), 1e-10)) (metrics.py:104-108, n values), the JL
dimension k (metrics.py:248) and -- unless the device ziggurat is selected --
the PCG64 normal stream R (metrics.py:272), streamed row-chunk by row-chunk.
"""

from __future__ import annotations

import ctypes
import os
import queue
import threading

import numpy as np

from . import _lib
from ._lib import GS_DEVICE, GS_HOST, Context, ptr

_ROW_CHUNK_BYTES = 64 << 20


def blas_threads_default() -> int:
    """OpenBLAS thread count NumPy would use for np.dot in this process.

    The reference's CG dot products are OpenBLAS ddot calls whose reduction
    order depends on it (n > 10000); GSPARSE_BLAS_THREADS overrides.  Clamped to
    OpenBLAS's MAX_THREADS (64 in NumPy's build), as OpenBLAS itself does."""
    return min(_blas_threads_requested(), OPENBLAS_MAX_THREADS)


OPENBLAS_MAX_THREADS = 64


def _blas_threads_requested() -> int:
    env = os.environ.get("GSPARSE_BLAS_THREADS")
    if env:
        return max(1, int(env))
    try:
        from threadpoolctl import threadpool_info

        for info in threadpool_info():
            if info.get("internal_api") == "openblas":
                return max(1, int(info.get("num_threads", 1)))
    except Exception:
        pass
    env = os.environ.get("OPENBLAS_NUM_THREADS")
    return max(1, int(env)) if env else 1


def jl_dim(n: int, epsilon: float) -> int:
    """metrics.py:248, evaluated with NumPy exactly as the reference does."""
    return max(int(24 * np.log(max(n, 2)) / (epsilon ** 2)), 1)


def aa_weights(indptr: np.ndarray) -> np.ndarray:
    """metrics.py:100-108 (adj_binary degrees -> c), NumPy ufuncs as the reference."""
    degrees = np.diff(indptr).astype(np.float64)
    log_degrees = np.log(degrees + 1)
    log_degrees = np.maximum(log_degrees, 1e-10)
    return 1.0 / np.sqrt(log_degrees)


def er_split(k: int, parts: int) -> list[int]:
    b = np.zeros(parts + 1, dtype=np.int64)
    _lib.check(_lib.lib().gs_er_split(k, parts, ptr(b)), "gs_er_split")
    return b.tolist()


class Engine:
    """Scorers over the graph resident in ``ctx``."""

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.n, self.nnz, self.symmetric = ctx.shape()
        self._indptr = None

    # -- helpers ------------------------------------------------------------
    def indptr(self) -> np.ndarray:
        if self._indptr is None:
            ip = np.empty(self.n + 1, dtype=np.int64)
            self.ctx.call("gs_graph_copy_csr", ptr(ip), None, None, GS_HOST)
            self._indptr = ip
        return self._indptr

    def _out(self, e0, e1, out):
        if out is None:
            return np.empty(e1 - e0, dtype=np.float64), GS_HOST
        return out, (GS_HOST if isinstance(out, np.ndarray) else GS_DEVICE)

    # -- scorers ------------------------------------------------------------
    def jaccard(self, e0: int = 0, e1: int | None = None, out=None):
        e1 = self.nnz if e1 is None else e1
        o, loc = self._out(e0, e1, out)
        self.ctx.call("gs_jaccard", e0, e1, ptr(o), loc)
        return o

    def jaccard_part(self, part: int, nparts: int, out=None):
        """Share `part` of `nparts` of the whole Jaccard vector (zeros elsewhere;
        the shares sum to jaccard()) -- gs_jaccard_part."""
        o, loc = self._out(0, self.nnz, out)
        self.ctx.call("gs_jaccard_part", part, nparts, ptr(o), loc)
        return o

    def jaccard_shares(self, nparts: int):
        """gs_jaccard_shares: (row_cut, owner_off), nparts + 1 values each -- the
        owner-pair shares of the sharded Jaccard (the same on every rank)."""
        rc = np.empty(nparts + 1, dtype=np.int64)
        oo = np.empty(nparts + 1, dtype=np.int64)
        self.ctx.call("gs_jaccard_shares", nparts, ptr(rc), ptr(oo))
        return rc, oo

    def jaccard_part_counts(self, part: int, nparts: int, out=None):
        """gs_jaccard_part_counts: |N(u) ∩ N(v)| of this part's owner pairs
        (uint32 numpy array, or the int32/uint32 device tensor ``out``)."""
        if not 0 <= part < nparts:
            raise ValueError(f"bad part {part} of {nparts}")
        _, oo = self.jaccard_shares(nparts)
        cnt = int(oo[part + 1] - oo[part])
        if out is None:
            o, loc = np.empty(cnt, dtype=np.uint32), GS_HOST
        else:
            if out.numel() < cnt:
                raise IndexError(f"counts buffer holds {out.numel()} < {cnt} values")
            o, loc = out, GS_DEVICE
        self.ctx.call("gs_jaccard_part_counts", part, nparts, ptr(o), loc)
        return o

    def jaccard_from_counts(self, nparts: int, counts, stride: int, out=None):
        """gs_jaccard_from_counts: every part's counts (part p at p * stride) ->
        the Jaccard score of every CSR entry."""
        cloc = GS_HOST if isinstance(counts, np.ndarray) else GS_DEVICE
        if cloc == GS_HOST:
            counts = np.ascontiguousarray(counts, dtype=np.uint32)
        if counts.shape[0] < nparts * stride:
            raise IndexError(f"counts hold {counts.shape[0]} < {nparts} x {stride} values")
        o, loc = self._out(0, self.nnz, out)
        self.ctx.call("gs_jaccard_from_counts", nparts, ptr(counts), stride, cloc, ptr(o), loc)
        return o

    # -- distributed Jaccard-T select (gs_jsel_*, include/gsparse.h) ---------
    JSEL_BINS, JSEL_PASSES = 8192, 5

    @staticmethod
    def _loc(a):
        if isinstance(a, np.ndarray):
            return GS_HOST
        return GS_DEVICE if a.is_cuda else GS_HOST

    @staticmethod
    def _need(a, count, dtypes, what):
        n = a.size if isinstance(a, np.ndarray) else a.numel()
        dt = a.dtype if isinstance(a, np.ndarray) else a.dtype
        if dt not in dtypes:
            raise TypeError(f"{what} must be one of {dtypes}, got {dt}")
        if n < count:
            raise IndexError(f"{what} holds {n} < {count} values")

    def jsel_begin(self, part: int, nparts: int, counts, num_keep: int, keep_lowest: bool, hist,
                   scores=None):
        """Keys (and, into ``scores``, the fp64 scores) of this part's owner pairs and the
        first weighted histogram into ``hist`` (JSEL_BINS int64/uint64 values)."""
        import torch

        _, oo = self.jaccard_shares(nparts)
        np_ = int(oo[part + 1] - oo[part])
        self._need(counts, np_, (np.uint32, np.int32, torch.int32), "counts")
        self._need(hist, self.JSEL_BINS, (np.uint64, np.int64, torch.int64), "hist")
        if self._loc(hist) != GS_DEVICE:
            raise ValueError("hist must be a device tensor (the ranks all-reduce it there)")
        sloc = GS_HOST
        if scores is not None:
            self._need(scores, np_, (np.float64, torch.float64), "scores")
            sloc = self._loc(scores)
        self.ctx.call("gs_jsel_begin", int(part), int(nparts), ptr(counts), self._loc(counts),
                      int(num_keep), int(bool(keep_lowest)), ptr(hist), ptr(scores), sloc)
        self._jsel_pairs = np_
        return np_

    def jsel_step(self, hist) -> int:
        """One pass of the select on the all-reduced ``hist``; returns the passes left."""
        left = ctypes.c_int(0)
        self.ctx.call("gs_jsel_step", ptr(hist), ctypes.byref(left))
        return left.value

    def jsel_result(self):
        """(cut, #beyond, #tied, #tied positions on this rank)."""
        cut, nb, nt, mine = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.call("gs_jsel_result", ctypes.byref(cut), ctypes.byref(nb), ctypes.byref(nt),
                      ctypes.byref(mine))
        return cut.value, nb.value, nt.value, mine.value

    def jsel_tie_positions(self, out):
        """This rank's tied CSR positions into ``out`` (int64)."""
        import torch

        self._need(out, 0, (np.int64, torch.int64), "positions")
        n = out.size if isinstance(out, np.ndarray) else out.numel()
        self.ctx.call("gs_jsel_tie_positions", ptr(out), int(n), self._loc(out))
        return out

    def jsel_keep(self, tie_pos, ntie: int, need: int, out):
        """2-bit keep codes of this part's pairs (bit 0 owner entry, bit 1 reverse entry),
        four pairs per byte, into ``out`` (uint8, >= ceil(pairs / 4) bytes)."""
        import torch

        np_ = getattr(self, "_jsel_pairs", 0)
        self._need(out, (np_ + 3) // 4, (np.uint8, torch.uint8), "keep")
        tloc = GS_HOST
        if tie_pos is not None:
            self._need(tie_pos, ntie, (np.int64, torch.int64), "tie positions")
            tloc = self._loc(tie_pos)
        self.ctx.call("gs_jsel_keep", ptr(tie_pos), int(ntie), tloc, int(need), ptr(out), self._loc(out))
        return out

    def jsel_mask(self, nparts: int, keep_all, stride: int, out):
        """Every part's keep codes (part p's from byte p * stride) -> the CSR keep mask (uint8)."""
        import torch

        self._need(keep_all, nparts * stride, (np.uint8, torch.uint8), "keep_all")
        self._need(out, self.nnz, (np.uint8, torch.uint8, torch.bool), "mask")
        self.ctx.call("gs_jsel_mask", int(nparts), ptr(keep_all), int(stride), self._loc(keep_all),
                      ptr(out), self._loc(out))
        return out

    def adamic_adar(self, e0: int = 0, e1: int | None = None, out=None, c=None):
        e1 = self.nnz if e1 is None else e1
        if c is None:
            c = np.ascontiguousarray(aa_weights(self.indptr()))
        o, loc = self._out(e0, e1, out)
        cloc = GS_HOST if isinstance(c, np.ndarray) else GS_DEVICE
        self.ctx.call("gs_adamic_adar", ptr(c), cloc, e0, e1, ptr(o), loc)
        return o

    def degree(self, e0: int = 0, e1: int | None = None, out=None):
        e1 = self.nnz if e1 is None else e1
        o, loc = self._out(e0, e1, out)
        self.ctx.call("gs_degree", e0, e1, ptr(o), loc)
        return o

    def feature_cosine(self, x, e0: int = 0, e1: int | None = None, out=None):
        """x: (n, f) float32/float64 numpy array or CUDA torch tensor."""
        e1 = self.nnz if e1 is None else e1
        if isinstance(x, np.ndarray):
            xloc = GS_HOST
            x = np.ascontiguousarray(x)
            dt = x.dtype
        else:
            xloc = GS_DEVICE if x.is_cuda else GS_HOST
            x = x.contiguous()
            if xloc == GS_HOST:
                x = x.numpy()
                dt = x.dtype
            else:
                import torch

                dt = {torch.float32: np.dtype(np.float32),
                      torch.float64: np.dtype(np.float64)}.get(x.dtype)
        if x.ndim != 2 or x.shape[0] != self.n:
            raise ValueError(f"features must be ({self.n}, f), got {tuple(x.shape)}")
        o, loc = self._out(e0, e1, out)
        if dt == np.float32:
            self.ctx.call("gs_feature_cosine_f32", ptr(x), int(x.shape[1]), xloc, e0, e1, ptr(o), loc)
        elif dt == np.float64:
            self.ctx.call("gs_feature_cosine_f64", ptr(x), int(x.shape[1]), xloc, e0, e1, ptr(o), loc)
        else:
            raise NotImplementedError(f"feature_cosine supports float32/float64 features, got {dt}")
        return o

    # -- ApproxER -----------------------------------------------------------
    def er_prepare(self, k: int, reg: float = 1e-6) -> int:
        m = ctypes.c_int64(0)
        self.ctx.call("gs_er_prepare", k, reg, ctypes.byref(m))
        self.k = k
        self.m = m.value
        return self.m

    def er_project_host(self, rng: np.random.Generator, k: int, cols=None):
        """Stream R = rng.standard_normal((m, k)) row-chunk by row-chunk (identical
        NumPy stream, verified chunk-invariant) into Y = B @ (R / sqrt(k)),
        generating chunk i+1 on a worker thread while chunk i is projected.
        cols = (c0, c1): form only Y[:, c0:c1] (a rank's JL columns)."""
        c0, c1 = cols if cols is not None else (0, k)
        m = self.m
        sqrt_k = float(np.sqrt(k))
        rows = max(1, _ROW_CHUNK_BYTES // (8 * k))
        q: queue.Queue = queue.Queue(maxsize=2)

        def producer():
            for e0 in range(0, m, rows):
                e1 = min(m, e0 + rows)
                q.put((e0, e1, rng.standard_normal((e1 - e0, k))))
            q.put(None)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        while True:
            item = q.get()
            if item is None:
                break
            e0, e1, raw = item
            self.ctx.call("gs_er_project_rows_cols", e0, e1, ptr(raw), GS_HOST, sqrt_k, c0, c1)
        th.join()

    def er_project_device(self, rng: np.random.Generator, k: int, cols=None):
        """The same R drawn on the device (PCG64 + NumPy's ziggurat); cols = (c0, c1):
        every normal is parsed, only R[:, c0:c1] is stored and projected."""
        c0, c1 = cols if cols is not None else (0, k)
        st = rng.bit_generator.state
        if st.get("bit_generator") != "PCG64":
            raise NotImplementedError("device ziggurat supports the PCG64 bit generator")
        s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
        m64 = (1 << 64) - 1
        if st.get("has_uint32"):
            raise NotImplementedError("PCG64 state with a buffered uint32")
        self.ctx.call("gs_er_project_pcg64_cols", s >> 64, s & m64, inc >> 64, inc & m64,
                      float(np.sqrt(k)), c0, c1)

    def er_solve(self, col0: int, col1: int, maxiter: int, rtol: float, blas_threads: int):
        self.ctx.call("gs_er_solve", col0, col1, maxiter, rtol, blas_threads)

    def er_scores(self, col0: int, col1: int, finalize: bool = True, e0: int = 0,
                  e1: int | None = None, out=None):
        e1 = self.nnz if e1 is None else e1
        o, loc = self._out(e0, e1, out)
        self.ctx.call("gs_er_scores", col0, col1, e0, e1, int(finalize), ptr(o), loc)
        return o

    def er_iterations(self) -> np.ndarray:
        it = np.empty(self.k, dtype=np.int32)
        self.ctx.call("gs_er_iterations", ptr(it), GS_HOST)
        return it

    def er_z(self, col0: int, col1: int) -> np.ndarray:
        """The solved Z columns [col0, col1) as an (n, col1 - col0) array (gs_er_copy_z)."""
        z = np.empty((self.n, col1 - col0), dtype=np.float64)
        self.ctx.call("gs_er_copy_z", col0, col1, ptr(z), GS_HOST)
        return z

    def approx_er(self, epsilon: float = 0.3, seed: int = 42, max_cg_iters: int = 500,
                  cg_tol: float = 1e-6, blas_threads: int | None = None,
                  rng_mode: str | None = None):
        """calculate_approx_effective_resistance_scores (metrics.py:178-298)."""
        rng = np.random.default_rng(seed)
        n = self.n
        k = jl_dim(n, epsilon)
        m = self.er_prepare(k)
        if m == 0:
            return np.zeros(self.nnz, dtype=np.float64)
        mode = rng_mode or os.environ.get("GSPARSE_ER_RNG", "device")
        if mode == "device":
            self.er_project_device(rng, k)
        else:
            self.er_project_host(rng, k)
        bt = blas_threads_default() if blas_threads is None else blas_threads
        self.er_solve(0, k, max_cg_iters, cg_tol, bt)
        return self.er_scores(0, k, True)

    # -- topology analytics (compute_topology_metrics, metrics.py:445-520) ----
    def common_neighbors(self, out=None):
        """gs_common_neighbors: |N(u) ∩ N(v)| per CSR entry (symmetric graph)."""
        o, loc = self._out(0, self.nnz, out)
        self.ctx.call("gs_common_neighbors", ptr(o), loc)
        return o

    def clustering(self, per_node: bool = False):
        """gs_clustering: nx.average_clustering of the resident (symmetric,
        self-loop-free) graph, bit-identical; optionally the per-node values."""
        avg = ctypes.c_double(0.0)
        cv = np.empty(max(self.n, 1), dtype=np.float64) if per_node else None
        self.ctx.call("gs_clustering", ctypes.byref(avg), ptr(cv) if cv is not None else None,
                      GS_HOST)
        return (avg.value, cv[: self.n]) if per_node else avg.value

    def components(self):
        """gs_components: (labels = smallest node id per component, count, largest)."""
        lab = np.empty(max(self.n, 1), dtype=np.int32)
        cnt, big = ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.call("gs_components", ptr(lab), GS_HOST, ctypes.byref(cnt), ctypes.byref(big))
        return lab[: self.n], cnt.value, big.value

    def fiedler(self, tol: float = 1e-12, max_iter: int = 300):
        """gs_fiedler: algebraic connectivity of the (connected) resident graph."""
        v, it = ctypes.c_double(0.0), ctypes.c_int32(0)
        self.ctx.call("gs_fiedler", float(tol), int(max_iter), ctypes.byref(v), ctypes.byref(it))
        self.fiedler_iterations = it.value
        return v.value

    # -- selection ------------------------------------------------------------
    def exact_er(self, out=None):
        """calculate_effective_resistance_scores (metrics.py:124-175) -- gs_exact_er:
        dense fp64-MFMA Newton-Schulz inverse of L + sum_C J_C/|C|."""
        o, loc = self._out(0, self.nnz, out)
        it = ctypes.c_int32(0)
        self.ctx.call("gs_exact_er", ptr(o), loc, ctypes.byref(it))
        self.exact_er_iterations = it.value
        return o

    def segment_argmax(self, scores: np.ndarray, src: np.ndarray, num_nodes: int) -> np.ndarray:
        """gs_segment_argmax: per node the column of its unique top score, -1 (no
        column) or -2 (np.argsort's order decides)."""
        scores = np.ascontiguousarray(scores, dtype=np.float64)
        src = np.ascontiguousarray(src, dtype=np.int64)
        pick = np.empty(max(num_nodes, 1), dtype=np.int64)
        self.ctx.call("gs_segment_argmax", ptr(scores), GS_HOST, int(scores.shape[0]), ptr(src),
                      GS_HOST, int(src.shape[0]), int(num_nodes), ptr(pick), GS_HOST)
        return pick[:num_nodes]

    def topk_mask(self, scores, num_edges: int, num_keep: int, keep_lowest: bool, out=None):
        """Device mask + (cut, #beyond, #tied) -- see gs_topk_mask.  ``scores``: a
        numpy array or a CUDA float64 tensor; ``out``: an optional CUDA uint8/bool
        tensor of >= num_edges elements that receives the mask on the device (then
        returned as is) instead of a host numpy bool array."""
        if isinstance(scores, np.ndarray):
            scores = np.ascontiguousarray(scores, dtype=np.float64)
            sloc = GS_HOST
        else:
            sloc = GS_DEVICE if scores.is_cuda else GS_HOST
            if sloc == GS_HOST:
                scores = np.ascontiguousarray(scores.numpy(), dtype=np.float64)
        nnz = int(scores.shape[0])
        if out is None:
            mask, mloc = np.zeros(num_edges, dtype=np.uint8), GS_HOST
        else:
            if not out.is_cuda or out.numel() < num_edges or out.element_size() != 1:
                raise ValueError("out must be a CUDA uint8/bool tensor of >= num_edges elements")
            mask, mloc = out, GS_DEVICE
        cut, nb, nt = ctypes.c_double(0), ctypes.c_int64(0), ctypes.c_int64(0)
        self.ctx.call("gs_topk_mask", ptr(scores), sloc, nnz, num_edges, num_keep,
                      int(keep_lowest), ptr(mask), mloc, ctypes.byref(cut), ctypes.byref(nb),
                      ctypes.byref(nt))
        return (mask.view(bool) if out is None else out), cut.value, nb.value, nt.value
