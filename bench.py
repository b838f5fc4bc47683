#!/usr/bin/env python3
"""Benchmark: scored edges/s of Jaccard + ApproxER (BASELINE.json metric).

Default workload (configs[1], N=1): the Roman-empire stand-in (roman_like:
n=22,662, E=65,854 directed CSR entries, 32,927 undirected edges, k=2,674 JL
columns, 500 CG iterations per column -- every column hits maxiter on this
chain-like graph, as on Roman-empire itself).  One step = Jaccard scores for
all E edges + the full ApproxER pipeline (PCG64/ziggurat normal stream on the
device -> Y = B R -> batched CG -> per-edge squared distances) with the CSR
resident in HBM.

N > 1 (torchrun, one process per GPU, RCCL over xGMI): the same problem
strong-scaled through gsparse.distributed -- Jaccard by contiguous CSR edge
ranges + all-gather of the scores, ApproxER by pairwise-tree blocks of JL
columns + all-gather of the per-edge partial sums combined in tree order (the
scores stay bit-identical to N=1).

Other workloads (not the default line): --workload rmat (Jaccard-T on
Graph500 R-MAT, configs[3]; --scale 22 by default), arxiv (configs[2]),
backbone (configs[4]), exact_er (the dense exact scorer, Cora size by
default, --xer-n for a Roman-like graph of that size; replicas at N > 1).

Prints ONE JSON line (rank 0) with roofline (dominant kernel, HIP events on
the library's stream) and cpu_baseline (the oracle's NumPy/SciPy restatement
of the reference path, bounded sample, timed on this host, rank 0 at N=1).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gnn-sparsification-research_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# MI355X dense fp64 matrix peak as AMD publishes it (the microarchitecture guide lists
# no fp64 figure); a register-only v_mfma_f64_16x16x4_f64 loop sustains 49-50 on the
# box (tools/mfma_f64_peak.hip, profiles/r01j_mfma_f64_peak.log).
FP64_MFMA_PEAK_TFS = 78.6
# fp64 VECTOR peak without contraction: 78.6 TFLOP/s counts an FMA as 2 flops; the CG
# must not contract (SciPy's separately rounded products), so its arithmetic roof is
# one fp64 op per lane-slot: 16 fp64 lanes per SIMD per clock x 1024 SIMDs x 2.4 GHz
FP64_VALU_PEAK_TFS = 39.3
SIMDS_PER_CU = 4


# profiler name -> kernel symbol prefix in the rocprofv3 summaries; "jaccard"
# is a pipeline of kernels (plan, light, hash classes, bitmap), summed per call
PMC_KERNEL = {"cg_res": "gs::k_cg_resident<", "cg_reg": "gs::k_cg_reg", "cg_pq": "gs::k_cg_pq<false", "cg_upd": "gs::k_cg_upd<",
              "jaccard": "gs::k_jac_", "metric_backbone": "gs::k_bb_",
              "cg_p": "gs::k_cg_p", "cg_spmv": "gs::k_spmv<"}
# kernels of a region that only its first call on a graph launches (the profiled run has
# one call; the timed steps repeat it): the symmetric Jaccard's plan -- row classes and
# per-class task lists, kept per (graph, part) -- and its algorithmic-byte sum (profiling
# only).  Their counters are not the timed call's.
PMC_FIRST_CALL = {"jaccard": ("k_jac_plan", "k_jac_mask", "k_jac_emit", "k_jac_bytes")}


sys.path.insert(0, os.path.join(ROOT, "tools"))
from provenance import source_hash  # noqa: E402

SRC_HASH = source_hash()
CU_COUNT, CLOCK_GHZ = 256, 2.4  # MI355X (MI355X_MICROARCH.md): issue-rate peaks below


def pmc_summary(workload: str):
    """The newest committed rocprofv3 PMC summary of this workload
    (profiles/*_<workload>_pmc_summary.json, tools/profile_bench.sh) that profiled
    THIS tree's libgsparse sources (its _meta.source_hash); counters of other code
    are never joined to this run's timings.  Returns (summary, file, note)."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{workload}_pmc_summary.json")))
    stale = None
    for f in reversed(files):
        with open(f) as fh:
            summ = json.load(fh)
        h = summ.get("_meta", {}).get("source_hash")
        if h == SRC_HASH:
            return summ, os.path.basename(f), None
        stale = stale or f"newest summary {os.path.basename(f)} profiled sources {h}, not {SRC_HASH}"
    return None, None, stale or f"no PMC summary of workload {workload!r}"


def kernel_counters(summ: dict, name: str, calls_per_step: float = 1.0):
    """Per-call counters of profiler entry `name`: the kernels of one call summed
    (pipelines: the plan kernel or the whole-column launch runs once per call).
    `calls_per_step`: calls of the region per bench step in the live run (the
    arxiv CG's batched kernels: one call per CG iteration)."""
    pre = PMC_KERNEL.get(name)
    if not summ or pre is None:
        return None
    hits = [(k, v) for k, v in summ.items()
            if k != "_meta" and (k.startswith("void " + pre) or k.startswith(pre))]
    if not hits:
        return None
    steps = summ.get("_meta", {}).get("calls_per_run")
    first = PMC_FIRST_CALL.get(name, ())
    skipped = sorted({k.split("(")[0].replace("void ", "") for k, _ in hits if any(f in k for f in first)})
    if steps and skipped:
        hits = [(k, v) for k, v in hits if not any(f in k for f in first)]
    if steps:
        # the profiled run made exactly `steps` bench steps (tools/profile_bench.sh: one
        # step, no box-order re-run), i.e. steps x calls_per_step calls of the region:
        # every kernel it launched, each weighted by its own launch count, divided by the
        # calls -- the timed call's kernel mix
        calls = steps * max(1.0, calls_per_step)
        out = {}
        for _, v in hits:
            for c, x in v.items():
                if c.endswith("_per_launch"):
                    key = c[: -len("_per_launch")]
                    out[key] = out.get(key, 0.0) + x * v.get("launches", 1) / calls
        out["kernels"] = len(hits)
        out["calls_per_run"] = calls
        out["first_call_only"] = skipped
        return out
    anchor = {"jaccard": "k_jac_plan", "metric_backbone": "k_bb_keep", "cg_reg": "k_cg_reg"}.get(name)
    if anchor and any(anchor in k for k, _ in hits):
        calls = max(1, max(v.get("launches", 1) for k, v in hits if anchor in k))
    else:
        hits = [max(hits, key=lambda kv: kv[1].get("launches", 0))]
        calls = hits[0][1].get("launches", 1)
    out = {}
    for _, v in hits:
        for c, x in v.items():
            if c.endswith("_per_launch"):
                out[c[: -len("_per_launch")]] = out.get(c[: -len("_per_launch")], 0.0) + \
                    x * v.get("launches", 1) / calls
    out["kernels"] = len(hits)
    return out


def make_roofline(name: str, avg_ms: float, bytes_per: float, launches: int, workload: str,
                  world: int, flops_per: float | None = None, steps: int | None = None) -> dict:
    """Roofline of the dominant kernel.  Headline (`achieved`, `frac`): measured
    HBM-side traffic -- rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per call of the same
    sources (FETCH_SIZE counts half of a wide stream on gfx950, WRITE_SIZE is exact:
    MI355X_MICROARCH.md) -- over this run's HIP-event launch time; a bound the
    kernel can reach.  `algorithmic`: SURVEY 8(d)'s bytes over the same time (above
    1 when the working set is re-read from LDS, registers or the Infinity Cache
    instead of HBM).  `on_chip`: issue rates from the SQ counters of the same
    summary (LDS array busy, VALU busy per SIMD, wave time spent waiting).

    `flops_per` (the CG solvers: SURVEY 8(d)'s SciPy operation count, 2 nnz(L_reg)
    + 12 n flops per column-iteration) makes the fp64 arithmetic roof the headline:
    those kernels keep r, x, p on chip by design, so HBM is not what bounds them
    (the measured HBM fraction stays, under `hbm`)."""
    alg = bytes_per / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    roof = {"kernel": name, "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None, "traffic": None, "avg_launch_ms": round(avg_ms, 5), "launches": launches,
            "basis": "measured traffic: rocprofv3 (2 x FETCH_SIZE + WRITE_SIZE) per call, same "
                     "sources, / live HIP-event launch time",
            "algorithmic": {"bytes_per_launch": bytes_per, "achieved": round(alg, 1),
                            "frac": round(alg / HBM_PEAK_GBS, 4),
                            "note": "SURVEY 8(d) algorithmic bytes; may exceed 1 (reuse on chip)"}}
    def fp64_headline(r, oc):
        # headline: the fp64 arithmetic roof; measured HBM traffic is the secondary view
        if not flops_per:
            return r
        tfs = flops_per / (avg_ms * 1e-3) / 1e12
        oc.update(fp64_tflops=round(tfs, 3), fp64_frac=round(tfs / FP64_VALU_PEAK_TFS, 4),
                  flops_per_launch=flops_per)
        r["hbm"] = {"achieved": r["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": r["frac"], "basis": r["basis"]}
        r.update(bound="fp64-valu", achieved=oc["fp64_tflops"], peak=FP64_VALU_PEAK_TFS,
                 unit="TFLOP/s", frac=oc["fp64_frac"],
                 basis="SURVEY 8(d) SciPy CG operation count (2 nnz(L_reg) + 12 n flops per "
                       "column-iteration) / live HIP-event launch time, against the fp64 VALU "
                       "peak without contraction")
        r.setdefault("on_chip", oc)
        return r

    if world > 1:  # the committed summaries are of 1-GPU runs (a rank launches a share)
        roof["basis"] = "no PMC at N > 1 (summaries are 1-GPU runs); see algorithmic"
        return fp64_headline(roof, {})
    summ, src, note = pmc_summary(workload)
    ctr = kernel_counters(summ, name, launches / steps if steps else 1.0) if summ else None
    if ctr is None or "FETCH_SIZE_KB" not in ctr or "WRITE_SIZE_KB" not in ctr:
        roof["basis"] = f"no counters for {name}: {note or src}; see algorithmic"
        return fp64_headline(roof, {})
    traffic = (2.0 * ctr["FETCH_SIZE_KB"] + ctr["WRITE_SIZE_KB"]) * 1024.0
    gbps = traffic / (avg_ms * 1e-3) / 1e9
    roof.update(achieved=round(gbps, 1), frac=round(gbps / HBM_PEAK_GBS, 4), traffic=round(traffic),
                traffic_source=f"{src} ({ctr['kernels']} kernel(s) per call)")
    if ctr.get("first_call_only"):
        roof["traffic_excludes"] = {"kernels": ctr["first_call_only"],
                                    "why": "launched by the first call on a graph only (the kept plan); "
                                           "the timed steps do not run them"}
    cyc = avg_ms * 1e-3 * CLOCK_GHZ * 1e9 * CU_COUNT  # CU-cycles of one launch
    oc = {}
    if "SQ_INSTS_LDS" in ctr:
        # LDS array cycles: 2 per conflict-free ds_read_b64 wave-instruction (the
        # kernels' dominant LDS op; MI355X_MICROARCH.md LDS table) + the measured
        # bank-conflict cycles, against one LDS array per CU
        busy = 2.0 * ctr["SQ_INSTS_LDS"] + ctr.get("SQ_LDS_BANK_CONFLICT", 0.0)
        oc["lds_busy_frac"] = round(busy / cyc, 4)
    if "SQ_ACTIVE_INST_VALU" in ctr:
        # VALU busy: SQ_ACTIVE_INST_VALU counts quad-cycles (summed over waves) in which a
        # wave executes VALU; a SIMD executes one wave's VALU at a time, so the bound is
        # the SIMDs' quad-cycles, 4 SIMDs per CU x CU-cycles / 4 (MI355X_MICROARCH.md
        # constants table: SQ_* count quad-cycles)
        oc["valu_busy_frac"] = round(ctr["SQ_ACTIVE_INST_VALU"] / (SIMDS_PER_CU * cyc / 4.0), 4)
    if "SQ_INSTS_VALU" in ctr:
        oc["valu_insts_per_launch"] = ctr["SQ_INSTS_VALU"]
    if "SQ_WAIT_ANY" in ctr and ctr.get("SQ_WAVE_CYCLES"):
        oc["wave_wait_frac"] = round(ctr["SQ_WAIT_ANY"] / ctr["SQ_WAVE_CYCLES"], 4)
    if oc:
        oc["source"] = src
        roof["on_chip"] = oc
    fp64_headline(roof, oc)
    if oc:
        # the nearest on-chip throughput bound (LDS array, VALU issue, fp64 arithmetic)
        oc["frac"] = max(oc.get("lds_busy_frac", 0.0), oc.get("valu_busy_frac", 0.0),
                         oc.get("fp64_frac", 0.0))
    return roof


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_info():
    """CPU model and logical CPU count of the box (state the cores)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"cpu_model": model, "logical_cpus": os.cpu_count()}


def emit(result):
    """The one JSON line; the CPU baseline names the host it ran on."""
    if isinstance(result.get("cpu_baseline"), dict):
        result["cpu_baseline"]["host"] = host_info()
    print(json.dumps(result), flush=True)


def host_cores() -> int:
    """CPU threads this process is granted: $OMP_NUM_THREADS when set (the GPU box
    sets it to its share of the host, 16 of 256), capped at the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(env))) if env and env.isdigit() else aff


def cpu_baseline_roman(ei, n, sample_cols, threads, all_cores_cols=16):
    """The reference algorithm restated with identical NumPy/SciPy calls
    (oracle/gsparse_oracle.py), timed on a bounded sample of the same
    workload: full Jaccard (A@A + gather, metrics.py:43-62), full R stream and
    Y = B @ R (metrics.py:272-275), SciPy CG on `sample_cols` of the k columns
    (metrics.py:284-289) extrapolated by k/sample_cols, and the diff^2 row sums
    (metrics.py:292-293) extrapolated from 64 columns.  The headline uses
    `threads` OpenBLAS threads (1: the fastest for this CG); the same pipeline
    with every core this process may use is reported beside it (`all_cores`,
    CG on `all_cores_cols` columns)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    from threadpoolctl import threadpool_limits

    import gsparse_oracle as O

    ip, ix, d = O.canonical_csr(ei, n)
    adj = sp.csr_matrix((d, ix, ip), shape=(n, n))

    def run(th, cols):
        with threadpool_limits(limits=th, user_api="blas"):
            t0 = time.perf_counter()
            ab = (adj > 0).astype(np.float64)
            deg = np.asarray(ab.sum(axis=1)).flatten()
            inter = ab @ ab
            rows, cols_ = ab.nonzero()
            ic = np.asarray(inter[rows, cols_]).flatten()
            uni = deg[rows] + deg[cols_] - ic
            _ = np.divide(ic, uni, out=np.zeros_like(ic), where=uni > 0)
            t_jac = time.perf_counter() - t0
            t0 = time.perf_counter()
            Y, m, kk = O.approx_er_projection(ip, ix, n)
            L = O.laplacian_reg(ip, ix, d, n)
            t_proj = time.perf_counter() - t0
            t0 = time.perf_counter()
            for i in range(cols):
                spla.cg(L, Y[:, i], maxiter=500, rtol=1e-6)
            t_cg = (time.perf_counter() - t0) * kk / cols
            t0 = time.perf_counter()
            Z = np.zeros((n, 64))
            diff = Z[rows] - Z[cols_]
            _ = np.sum(diff ** 2, axis=1)
            t_fin = (time.perf_counter() - t0) * kk / 64
        total = t_jac + t_proj + t_cg + t_fin
        return total, (f"full Jaccard ({t_jac:.3f}s) + full R/Y projection ({t_proj:.2f}s) + SciPy CG "
                       f"on {cols}/{kk} columns x500 iters extrapolated ({t_cg:.1f}s) + "
                       f"diff^2 sum extrapolated ({t_fin:.2f}s); OpenBLAS threads={th}")

    total, sample = run(threads, sample_cols)
    res = {"value": float(len(ix) / total), "unit": "scored edges/s", "cores": int(threads),
           "kind": "port", "sample": sample, "seconds_extrapolated": round(total, 3)}
    allc = host_cores()
    if allc > threads:
        t_all, s_all = run(allc, all_cores_cols)
        res["all_cores"] = {"value": float(len(ix) / t_all), "cores": allc, "sample": s_all,
                            "seconds_extrapolated": round(t_all, 3)}
    return res


def cpu_baseline_arxiv(ei, n, cg_cols=16, row_div=64, diff_cols=64):
    """configs[2] CPU baseline: the reference's calls (metrics.py:17-64, 232-297) restated
    with the same NumPy/SciPy operations (oracle/gsparse_oracle.py), 1 OpenBLAS thread,
    on a bounded sample -- the reference itself would allocate R (m x k = 30 GB) and
    diff (E x k = 60 GB) at this size:
    * Jaccard in full (A@A, gather, divide);
    * R = standard_normal((m, k)) / sqrt(k) for m/row_div rows, and Y = B @ R for those
      rows, both x row_div;
    * SciPy CG (maxiter 500, rtol 1e-6) on `cg_cols` columns x k/cg_cols; their
      right-hand sides are B @ N(0,1)/sqrt(k) columns of an independent draw (same
      distribution, so the same iteration counts; timing only);
    * diff = Z[rows] - Z[cols] and its row sums on `diff_cols` columns x k/diff_cols."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import scipy.sparse as sp
    import scipy.sparse.linalg as spla
    from threadpoolctl import threadpool_limits

    import gsparse_oracle as O

    ip, ix, d = O.canonical_csr(ei, n)
    adj = sp.csr_matrix((d, ix, ip), shape=(n, n))
    rows = O.csr_rows(ip)
    k = O.jl_dim(n)
    with threadpool_limits(limits=1, user_api="blas"):
        t0 = time.perf_counter()
        ab = (adj > 0).astype(np.float64)
        deg = np.asarray(ab.sum(axis=1)).flatten()
        inter = ab @ ab
        rr, cc = ab.nonzero()
        ic = np.asarray(inter[rr, cc]).flatten()
        uni = deg[rr] + deg[cc] - ic
        _ = np.divide(ic, uni, out=np.zeros_like(ic), where=uni > 0)
        t_jac = time.perf_counter() - t0
        mask = rows < ix
        u_e, v_e = rows[mask], ix[mask].astype(np.int64)
        m = len(u_e)
        ms = max(1, m // row_div)
        rng = np.random.default_rng(42)
        B = sp.csr_matrix((np.concatenate([np.ones(m), -np.ones(m)]),
                           (np.concatenate([u_e, v_e]), np.concatenate([np.arange(m), np.arange(m)]))),
                          shape=(n, m))
        t0 = time.perf_counter()
        Rs = rng.standard_normal((ms, k)) / np.sqrt(k)
        t_r = (time.perf_counter() - t0) * m / ms
        # the sampled edges' rows of B only (the full product's n x k output is written
        # once, not once per sample)
        Bs = B[:, :ms].tocsr()
        Bs = Bs[np.flatnonzero(np.diff(Bs.indptr))]
        t0 = time.perf_counter()
        _ = Bs @ Rs
        t_y = (time.perf_counter() - t0) * m / ms
        del Rs
        Y = B @ (np.random.default_rng(7).standard_normal((m, cg_cols)) / np.sqrt(k))
        L = O.laplacian_reg(ip, ix, d, n)
        t0 = time.perf_counter()
        its = 0
        for i in range(cg_cols):
            cnt = [0]

            def cb(_x, c=cnt):
                c[0] += 1
            spla.cg(L, Y[:, i], maxiter=500, rtol=1e-6, callback=cb)
            its += cnt[0]
        t_cg = (time.perf_counter() - t0) * k / cg_cols
        Z = np.zeros((n, diff_cols))
        t0 = time.perf_counter()
        diff = Z[rows] - Z[ix]
        _ = np.sum(diff ** 2, axis=1)
        t_fin = (time.perf_counter() - t0) * k / diff_cols
    total = t_jac + t_r + t_y + t_cg + t_fin
    return {"value": float(len(ix) / total), "unit": "scored edges/s", "cores": 1, "kind": "port",
            "sample": (f"full Jaccard ({t_jac:.2f}s) + R stream of {ms}/{m} rows x{m / ms:.0f} "
                       f"({t_r:.1f}s) + B@R of those rows x{m / ms:.0f} ({t_y:.1f}s) + SciPy CG on "
                       f"{cg_cols}/{k} columns ({its / cg_cols:.0f} iterations per column) x{k / cg_cols:.0f} "
                       f"({t_cg:.1f}s) + diff^2 sums on {diff_cols} columns x{k / diff_cols:.0f} "
                       f"({t_fin:.1f}s); OpenBLAS threads=1; the reference would hold R "
                       f"({8 * m * k / 1e9:.0f} GB) and diff ({8 * len(ix) * k / 1e9:.0f} GB) at once"),
            "seconds_extrapolated": round(total, 2)}


def cpu_baseline_rmat(ip, ix, n, scale, merge_steps=3e9, spgemm_scale=15):
    """configs[3] CPU baseline, two legs on this host's cores (1 thread each):
    (1) the per-edge sorted-list merge restated in C (oracle.c, the same counts and
    division as metrics.py:43-62) on the rows of a prefix holding ~merge_steps merge
    steps, extrapolated by the whole graph's sum of (d_u + d_v);
    (2) the reference's own SpGEMM Jaccard (A_bin @ A_bin, gather, divide:
    metrics.py:43-62) on the full R-MAT-`spgemm_scale` graph -- the largest that
    runs in ~15 s here (R-MAT-22 would materialise ~1e11 two-hop pairs) --
    extrapolated to this graph by the SpGEMM's work sum_w d_w^2."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes

    import scipy.sparse as sp
    from threadpoolctl import threadpool_limits

    import gsparse_oracle as O
    from gsparse import graphs

    deg = np.diff(ip)
    rows = np.repeat(np.arange(n, dtype=np.int64), deg)
    work = deg[rows] + deg[ix]
    cw = np.cumsum(np.bincount(rows, weights=work, minlength=n))
    r1 = int(min(n, np.searchsorted(cw, merge_steps) + 1))
    tp, ti = O.transpose(ip, ix, n)
    out = np.zeros(len(ix), dtype=np.float64)
    t0 = time.perf_counter()
    O.lib().oracle_jaccard_rows(O._p(ip, O._i64p), O._p(ix, O._i32p), O._p(tp, O._i64p),
                                O._p(ti, O._i32p), ctypes.c_int64(0), ctypes.c_int64(r1),
                                O._p(out, O._f64p))
    t_merge = time.perf_counter() - t0
    frac = float(cw[r1 - 1]) / float(cw[-1])
    merge_total = t_merge / frac
    # (2) reference SpGEMM on a smaller R-MAT, scaled by sum_w d_w^2
    ei_s = graphs.rmat(spgemm_scale, 8, seed=0)
    ns = 1 << spgemm_scale
    ips, ixs, ds = O.canonical_csr(ei_s, ns)
    adj = sp.csr_matrix((ds, ixs, ips), shape=(ns, ns))
    with threadpool_limits(limits=1, user_api="blas"):
        t0 = time.perf_counter()
        ab = (adj > 0).astype(np.float64)
        dg = np.asarray(ab.sum(axis=1)).flatten()
        inter = ab @ ab
        rr, cc = ab.nonzero()
        ic = np.asarray(inter[rr, cc]).flatten()
        uni = dg[rr] + dg[cc] - ic
        _ = np.divide(ic, uni, out=np.zeros_like(ic), where=uni > 0)
        t_sp = time.perf_counter() - t0
    w_small = float(np.sum(np.diff(ips).astype(np.float64) ** 2))
    w_big = float(np.sum(deg.astype(np.float64) ** 2))
    spgemm_total = t_sp * w_big / w_small
    best = min(merge_total, spgemm_total)
    return {"value": float(len(ix) / best), "unit": "scored edges/s", "cores": 1, "kind": "port",
            "sample": (f"per-edge merge (oracle.c) on rows [0, {r1}) = {frac:.3%} of the merge steps: "
                       f"{t_merge:.1f}s -> {merge_total:.0f}s for RMAT-{scale}; reference SpGEMM "
                       f"(metrics.py:43-62) on the full RMAT-{spgemm_scale} ({len(ixs)} edges): "
                       f"{t_sp:.1f}s -> {spgemm_total:.0f}s for RMAT-{scale} by sum d^2 "
                       f"({w_big:.3g} / {w_small:.3g}); value = the faster leg"),
            "seconds_extrapolated": round(best, 1),
            "legs": {"merge_restated_s": round(merge_total, 1),
                     "reference_spgemm_s": round(spgemm_total, 1)}}


def cpu_baseline_backbone(ei, n, w, n_src=16, seed=0):
    """The reference's algorithm (metric_backbone.py:86-111: NetworkX Dijkstra
    from every node over the undirected u<v graph, then the per-column test) on
    `n_src` sampled source rows, extrapolated by (#rows with columns)/n_src."""
    import networkx as nx

    ei = np.asarray(ei)
    m = ei[0] < ei[1]
    G = nx.Graph()
    G.add_nodes_from(range(n))
    for a, b, x in zip(ei[0][m].tolist(), ei[1][m].tolist(), np.asarray(w)[m].tolist()):
        if G.has_edge(a, b):
            if x < G[a][b]["weight"]:
                G[a][b]["weight"] = x
        else:
            G.add_edge(a, b, weight=x)
    rows = np.unique(ei[0])
    rng = np.random.default_rng(seed)
    sample = rng.choice(rows, min(n_src, len(rows)), replace=False)
    t0 = time.perf_counter()
    for u in sample.tolist():
        nx.single_source_dijkstra_path_length(G, u, weight="weight")
    t = time.perf_counter() - t0
    total = t * len(rows) / len(sample)
    return {"value": float(ei.shape[1] / total), "unit": "scored edges/s", "cores": 1,
            "kind": "port",
            "sample": f"NetworkX Dijkstra from {len(sample)} of {len(rows)} source rows "
                      f"({t:.2f}s), extrapolated to all rows ({total:.0f}s)"}


def bench_backbone(args, world, rank, local_rank, dev, dist):
    """configs[4]: metric_backbone prune on R-MAT (default scale 18) or the
    Roman-like graph; costs = _scores_to_cost(Jaccard) as
    sparsify_metric_backbone passes them (core.py:251-279).  One step = the
    whole prune (graph build, witnesses, certificates, bounded searches) on
    device-resident columns; N > 1 runs the staged form (gsparse.distributed.
    sharded_backbone): landmark searches split over the ranks, witnesses and
    certificates by column range, searches by source in ranges of the ascending-count
    order, with all-reduces of the labels and column states between the stages."""
    import ctypes

    from gsparse import graphs
    from gsparse._lib import GS_DEVICE, Context
    from gsparse.core import GraphSparsifier
    from gsparse.data import Data
    from gsparse.distributed import Comm

    t_gen = time.perf_counter()
    if args.bb_graph == "roman":
        ei, n = graphs.roman_like(), 22_662
        wl = "configs[4] metric backbone, Roman-like, Jaccard costs"
    else:
        ei, n = graphs.rmat(args.bb_scale, 8, seed=0), 1 << args.bb_scale
        wl = f"configs[4] metric backbone, RMAT-{args.bb_scale}, Jaccard costs"
    t_gen = time.perf_counter() - t_gen
    E = ei.shape[1]
    sp_ = GraphSparsifier(Data(edge_index=torch.from_numpy(ei), num_nodes=n), f"cuda:{local_rank}")
    cost = sp_._scores_to_cost(sp_.compute_scores("jaccard"), "jaccard")[:E]
    ctx = Context(local_rank)
    src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
    dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
    w = torch.from_numpy(np.ascontiguousarray(cost, dtype=np.float64)).to(dev)
    keep = torch.empty(E, dtype=torch.uint8, device=dev)
    comm = Comm(device=dev) if world > 1 else None
    relax = ctypes.c_int64(0)
    if comm is not None:
        from gsparse.distributed import sharded_backbone
        from gsparse.metric_backbone import BackboneStages

        stages = BackboneStages(ctx)
        ei_d = torch.stack([src, dst])

    def step():
        if comm is not None:
            # staged over the ranks (gs_bb_*): landmarks split, columns by range, searches
            # by source in ranges of the ascending-count order, state all-reduces between
            return sharded_backbone(comm, ei_d, n, w, 1e-9, stages=stages, keep_out=keep)
        ctx.call("gs_metric_backbone", n, E, src.data_ptr(), dst.data_ptr(), w.data_ptr(),
                 w.numel(), GS_DEVICE, 1e-9, keep.data_ptr(), GS_DEVICE, ctypes.byref(relax))
        return keep

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.profile(True)
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if dist.get_backend() != "nccl":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kept = int((out != 0).sum().item())
    roofline = None
    if prof and "metric_backbone" in prof:
        p = prof["metric_backbone"]
        key = f"backbone-{args.bb_graph}" + (str(args.bb_scale) if args.bb_graph == "rmat" else "")
        roofline = make_roofline("metric_backbone", p["ms"] / p["launches"], p["bytes"] / p["launches"],
                                 p["launches"], key, world, steps=args.steps)
        roofline["relaxations_per_launch_rank0"] = relax.value if comm is None else stages.relax
    result = {
        "metric": "scored edges/sec (metric backbone)", "value": round(E * args.steps / elapsed, 1),
        "unit": "scored edges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": wl, "n": n, "E": E, "kept": kept,
                   "parallelism": f"staged sources/{world}" if world > 1 else "1 GPU",
                   "graph_gen_s": round(t_gen, 2)},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_backbone(ei, n, cost)
    if rank == 0:
        emit(result)
    if dist:
        dist.destroy_process_group()


def cpu_baseline_exact_er(indptr, indices, data, n, max_n=4000):
    """The reference's calculate_effective_resistance_scores (metrics.py:124-175:
    dense pinv of L + 1e-10 I by SVD) restated in NumPy (oracle.exact_er,
    lifted=False, bit-identical to the reference's golden vectors) on this graph,
    or -- above max_n nodes -- on its first max_n-node induced subgraph with the
    time scaled by (n / max_n)^3."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import scipy.sparse as sp

    import gsparse_oracle as O

    try:
        from threadpoolctl import threadpool_info

        cores = max(int(i.get("num_threads", 1)) for i in threadpool_info()
                    if i.get("user_api") == "blas")
    except Exception:
        cores = int(os.environ.get("OMP_NUM_THREADS", "1"))
    m = min(n, max_n)
    a = sp.csr_matrix((data, indices, indptr), shape=(n, n))[:m, :m].tocsr()
    t0 = time.perf_counter()
    O.exact_er(a.indptr, a.indices, a.data, m, lifted=False)
    t = time.perf_counter() - t0
    total = t * (n / m) ** 3
    what = "this graph" if m == n else f"the first {m} nodes' subgraph, x(n/{m})^3"
    return {"value": float(len(indices) / total), "unit": "scored edges/s", "cores": cores,
            "kind": "port",
            "sample": f"NumPy pinv(L + 1e-10 I) as metrics.py:159-173 on {what} "
                      f"({t:.2f}s measured, {total:.1f}s for the graph); BLAS threads={cores}"}


def bench_topology(args, world, rank, local_rank, dev, dist):
    """compute_topology_metrics (metrics.py:445-520) on the
    Roman-like graph (default) or the Cora-size Chung-Lu graph (--xer-n 2708):
    edges, degrees, clustering, components and the algebraic connectivity, one
    step = the whole call.  CPU baseline: the reference's NetworkX calls
    (oracle.topology_metrics).  Replicas only (per-graph analytics)."""
    from gsparse import graphs
    from gsparse.metrics import compute_topology_metrics

    import scipy.sparse as sp

    if args.xer_n == 2708:
        n, ei, wl = 2_708, graphs.chung_lu(), "topology metrics, Cora-size Chung-Lu"
    else:
        n = args.xer_n or 22_662
        ei = graphs.roman_like(n=n, m=int(n * 32_927 / 22_662), seed=0)
        wl = f"topology metrics, Roman-like n={n}"
    A = sp.csr_matrix((np.ones(ei.shape[1]), (ei[0], ei[1])), shape=(n, n))
    A.sum_duplicates()
    from gsparse.metrics import _scratch_context

    ctx = _scratch_context()
    for _ in range(args.warmup):
        res = compute_topology_metrics(A)
    torch.cuda.synchronize(dev)
    ctx.profile(True)
    ctx.profile_reset()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = compute_topology_metrics(A)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    roofline = None
    if prof and "exact_er_dgemm" in prof:
        p = prof["exact_er_dgemm"]
        avg_ms = p["ms"] / p["launches"]
        fl = p["bytes"] / p["launches"]
        achieved = fl / (avg_ms * 1e-3) / 1e12
        roofline = {"kernel": "k_chol_diag + k_tile_mm (grounded Cholesky and L^-1 for L^+)",
                    "bound": "mfma", "achieved": round(achieved, 2), "peak": FP64_MFMA_PEAK_TFS,
                    "unit": "TFLOP/s", "frac": round(achieved / FP64_MFMA_PEAK_TFS, 4),
                    "traffic": None, "avg_launch_ms": round(avg_ms, 4), "flops_per_launch": fl,
                    "launches": p["launches"]}
    result = {
        "metric": "topology-metric calls/sec (compute_topology_metrics)",
        "value": round(world * args.steps / elapsed, 3), "unit": "calls/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": wl, "n": n, "E": int(A.nnz),
                   "parallelism": f"{world} replicas" if world > 1 else "1 GPU",
                   "result": {k: (float(v) if isinstance(v, (float, np.floating)) else int(v))
                              for k, v in res.items()}},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import gsparse_oracle as O

        t = time.perf_counter()
        O.topology_metrics(A)
        sec = time.perf_counter() - t
        result["cpu_baseline"] = {"value": round(1.0 / sec, 4), "unit": "calls/s", "cores": 1,
                                  "kind": "port",
                                  "sample": "the reference's NetworkX calls (average_clustering, "
                                            "connected_components, algebraic_connectivity "
                                            f"tracemin_lu), one full call: {sec:.2f} s"}
    if rank == 0:
        emit(result)


def bench_geodesic(args, world, rank, local_rank, dev, dist):
    """compute_geodesic_preservation (metrics.py:361-442) + verify_geodesic_preservation
    (metric_backbone.py:144-225) on the Roman-like graph: 500 sampled pairs,
    hop distances original vs the top-50% Jaccard subgraph, weighted (Jaccard
    cost) distances original vs the same subgraph; one step = both calls.
    CPU baseline: the reference's NetworkX calls (oracle.geodesic_preservation,
    oracle.verify_geodesic).  Replicas only."""
    from gsparse import graphs
    from gsparse.data import Data
    from gsparse.core import GraphSparsifier
    from gsparse.metrics import compute_geodesic_preservation
    from gsparse.metric_backbone import verify_geodesic_preservation

    import scipy.sparse as sp

    n = args.xer_n or 22_662
    ei = graphs.roman_like(n=n, m=int(n * 32_927 / 22_662), seed=0)
    data = Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    sp_ = GraphSparsifier(data, "cpu")
    scores = sp_.compute_scores("jaccard")
    cost = sp_._scores_to_cost(scores, "jaccard")
    _, keep = sp_.sparsify("jaccard", 0.5, return_mask=True)
    keep = keep.numpy()
    ei_s = ei[:, keep]
    sub = Data(edge_index=torch.from_numpy(ei_s), num_nodes=n)
    A = sp.csr_matrix((np.ones(ei.shape[1]), (ei[0], ei[1])), shape=(n, n))
    S = sp.csr_matrix((np.ones(ei_s.shape[1]), (ei_s[0], ei_s[1])), shape=(n, n))

    def step():
        a = compute_geodesic_preservation(A, S, n_samples=500)
        b = verify_geodesic_preservation(data, sub, cost, cost[keep], n_samples=500)
        return a, b

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    a, b = res
    result = {
        "metric": "geodesic-check calls/sec (compute_geodesic_preservation + verify_geodesic_preservation)",
        "value": round(world * args.steps / elapsed, 3), "unit": "calls/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": f"geodesic checks, Roman-like n={n}, top-50% Jaccard subgraph, 500 pairs",
                   "n": n, "E": int(ei.shape[1]), "kept": int(keep.sum()),
                   "parallelism": f"{world} replicas" if world > 1 else "1 GPU",
                   "result": {"preservation_ratio": float(a["preservation_ratio"]),
                              "violations": int(b["violations"]),
                              "unreachable_backbone": int(b["unreachable_backbone"])}},
        "roofline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import gsparse_oracle as O

        t = time.perf_counter()
        O.geodesic_preservation(A, S, n_samples=500)
        O.verify_geodesic(ei, cost, ei_s, cost[keep], n, n_samples=500)
        sec = time.perf_counter() - t
        result["cpu_baseline"] = {"value": round(1.0 / sec, 4), "unit": "calls/s", "cores": 1,
                                  "kind": "port",
                                  "sample": "the reference's NetworkX calls (shortest_path_length "
                                            f"hop + Dijkstra, 500 pairs each), one full step: {sec:.2f} s"}
    if rank == 0:
        emit(result)


def bench_exact_er(args, world, rank, local_rank, dev, dist):
    """calculate_effective_resistance_scores (metrics.py:124-175), the exact
    (dense) scorer the reference runs on small graphs: default Cora-size
    (Chung-Lu stand-in, n=2,708 / 5,278 edges, configs[0]'s graph size), or a
    Roman-like graph of --xer-n nodes.  One step = gs_exact_er end to end
    (components, grounding, blocked Cholesky + L^-1 on fp64 MFMA -- or
    Newton-Schulz with GSPARSE_XER_METHOD=ns -- and the per-edge read-out).
    Replicas only: every rank scores its own copy (the dense inverse does not
    shard without an exchange of X every step)."""
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.engine import Engine
    from gsparse.metrics import _prepare

    import scipy.sparse as sp

    if args.xer_n:
        n = args.xer_n
        ei = graphs.roman_like(n=n, m=int(n * 32_927 / 22_662), seed=0)
        wl = f"exact ER, Roman-like n={n}"
    else:
        n = 2_708
        ei = graphs.chung_lu()
        wl = "exact ER, Cora-size Chung-Lu (n=2,708, 5,278 undirected edges)"
    A = sp.csr_matrix((np.ones(ei.shape[1]), (ei[0], ei[1])), shape=(n, n))
    A.sum_duplicates()
    a, _ = _prepare(A)
    ctx = Context(local_rank)
    ctx.set_graph_csr(n, a.indptr, a.indices, a.data)
    eng = Engine(ctx)
    E = int(a.nnz)
    out = torch.empty(E, dtype=torch.float64, device=dev)

    def step():
        eng.exact_er(out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.profile(True)
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if dist.get_backend() != "nccl":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    roofline = None
    if prof and "exact_er_dgemm" in prof:
        p = prof["exact_er_dgemm"]
        avg_ms = p["ms"] / p["launches"]
        fl = p["bytes"] / p["launches"]  # executed flops per launch
        achieved = fl / (avg_ms * 1e-3) / 1e12
        ns = os.environ.get("GSPARSE_XER_METHOD") == "ns"
        roofline = {"kernel": "k_dgemm<true,64>" if ns else
                    "k_chol_diag + k_tile_mm (blocked Cholesky and L^-1, one profiled region)",
                    "bound": "mfma", "achieved": round(achieved, 2),
                    "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s",
                    "frac": round(achieved / FP64_MFMA_PEAK_TFS, 4), "traffic": None,
                    "avg_launch_ms": round(avg_ms, 4), "flops_per_launch": fl,
                    "launches": p["launches"]}
        if ns:
            roofline["newton_schulz_steps"] = eng.exact_er_iterations
        else:
            roofline["blocks_64"] = eng.exact_er_iterations
        if "exact_er_spmm" in prof:
            q = prof["exact_er_spmm"]
            qa = q["bytes"] / q["ms"] * 1e-6
            roofline["spmm"] = {"bound": "hbm", "achieved": round(qa, 1), "peak": HBM_PEAK_GBS,
                                "unit": "GB/s", "frac": round(qa / HBM_PEAK_GBS, 4),
                                "avg_launch_ms": round(q["ms"] / q["launches"], 4)}
    result = {
        "metric": "scored edges/sec (exact effective resistance)",
        "value": round(world * E * args.steps / elapsed, 1),
        "unit": "scored edges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": wl, "n": n, "E": E,
                   "parallelism": f"{world} replicas" if world > 1 else "1 GPU"},
        "roofline": roofline,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline_exact_er(a.indptr, a.indices, a.data, n)
    if rank == 0:
        emit(result)
    if dist:
        dist.destroy_process_group()


def bench_scorers(args, world, rank, local_rank, dev, dist):
    """configs[1] with every scorer: on the Roman-empire stand-in, one step =
    Jaccard (metrics.py:17-64), Adamic-Adar (:67-121), FeatCos on 300-d float32
    features (:301-358) and ApproxER (:178-298) over all E edges, inputs
    resident in HBM.  Per-scorer rooflines by SURVEY 8(d)'s algorithmic bytes
    (B_J, B_AA, B_F, B_ER); the line's roofline is the dominant kernel's.  CPU
    baseline: the oracle's NumPy restatements of Jaccard / AA / FeatCos (full)
    plus the ApproxER sample of the default line.  Replicas at N > 1."""
    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.engine import Engine, aa_weights, jl_dim

    ei, n, f = graphs.roman_like(), 22_662, 300
    x = graphs.features(n, f, seed=1)
    E = ei.shape[1]
    ctx = Context(local_rank)
    ctx.set_graph_edge_index(n, torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev),
                             torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev))
    eng = Engine(ctx)
    nnz = eng.nnz
    k = jl_dim(n, 0.3)
    indptr, indices, _ = ctx.csr()
    xd = torch.from_numpy(x).to(dev)
    cd = torch.from_numpy(np.ascontiguousarray(aa_weights(indptr))).to(dev)
    outs = [torch.empty(nnz, dtype=torch.float64, device=dev) for _ in range(4)]

    def step():
        eng.jaccard(0, nnz, out=outs[0])
        eng.adamic_adar(0, nnz, out=outs[1], c=cd)
        eng.feature_cosine(xd, 0, nnz, out=outs[2])
        rng = np.random.default_rng(42)
        eng.er_prepare(k)
        eng.er_project_device(rng, k)
        eng.er_solve(0, k, 500, 1e-6, args.blas_threads)
        eng.er_scores(0, k, True, out=outs[3])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.profile(True)
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    # SURVEY 8(d) algorithmic bytes (binarised degrees; the graph is symmetric)
    deg = np.diff(indptr).astype(np.float64)
    rows = np.repeat(np.arange(n), np.diff(indptr))
    b_j = 4.0 * float(np.sum(deg[rows] + deg[indices])) + 12.0 * nnz
    b_aa = b_j + 8.0 * float(np.sum(eng.common_neighbors()))
    b_f = 2.0 * f * 4 * nnz + 8.0 * nnz + 3.0 * n * f * 4

    def roof(names, by):
        ms = sum(prof[nm]["ms"] for nm in names if nm in prof)
        la = max((prof[nm]["launches"] for nm in names if nm in prof), default=0)
        if not la or ms <= 0:
            return None
        avg = ms / la
        ach = by / (avg * 1e-3) / 1e9
        return {"kernels": names, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(avg, 4),
                "algorithmic_bytes_per_launch": by}

    per = {"jaccard": roof(["jaccard"], b_j), "adamic_adar": roof(["adamic_adar"], b_aa),
           "feature_cosine": roof(["featcos_normalise", "featcos_edges"], b_f)}
    name = next((kk for kk in ("cg_reg", "cg_res") if kk in prof), None) or max(
        prof, key=lambda kk: prof[kk]["ms"])
    p = prof[name]
    roofline = make_roofline(name, p["ms"] / p["launches"], p["bytes"] / p["launches"], p["launches"],
                             "roman", world, steps=args.steps)
    result = {
        "metric": "scored edges/sec (Jaccard+AA+FeatCos+ApproxER)",
        "value": round(world * E * args.steps / elapsed, 1), "unit": "scored edges/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 2), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64 (FeatCos in f32, as the reference)",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": "configs[1] Roman-empire all scorers", "n": n, "E": E, "features": f,
                   "jl_k": k, "cg_maxiter": 500, "blas_threads_order": args.blas_threads,
                   "parallelism": f"{world} replicas" if world > 1 else "1 GPU"},
        "roofline": roofline, "scorer_rooflines": per,
        "kernels": {kk: {"launches": v["launches"], "ms": round(v["ms"], 3)} for kk, v in prof.items()},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import gsparse_oracle as O

        ip, ix, _ = O.canonical_csr(ei, n)
        t = time.perf_counter()
        O.adamic_adar(ip, ix)
        t_aa = time.perf_counter() - t
        t = time.perf_counter()
        O.feature_cosine(ip, ix, x)
        t_fc = time.perf_counter() - t
        base = cpu_baseline_roman(ei, n, args.cpu_sample_cols, 1)
        total = base["seconds_extrapolated"] + t_aa + t_fc
        result["cpu_baseline"] = {
            "value": float(E / total), "unit": "scored edges/s", "cores": 1, "kind": "port",
            "sample": f"AA ({t_aa:.2f}s) + FeatCos ({t_fc:.2f}s) in full + " + base["sample"],
            "seconds_extrapolated": round(total, 3)}
    if rank == 0:
        emit(result)


def spawn_ranks(n: int, rehearse: bool) -> None:
    """`bench.py --gpus N` without a launcher: start N ranks (one per GPU) with
    torch.distributed.run as a child process and exit with its status -- the
    driver's own launch (torchrun + WORLD_SIZE) skips this.  Fails loudly when
    fewer than N GPUs are visible (GSPARSE_REHEARSE=1: ranks share them)."""
    import socket
    import subprocess

    visible = torch.cuda.device_count()
    if n > visible and not rehearse:
        raise SystemExit(f"bench.py: --gpus {n} needs {n} GPUs, {visible} visible")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    cmd += sys.argv[1:]
    log(f"bench.py: launching {n} ranks: {' '.join(cmd)}")
    sys.exit(subprocess.call(cmd))


def check_ranks(dist, world: int, local_rank: int, rehearse: bool) -> None:
    """Every rank is up, and (unless rehearsing) each drives its own GPU."""
    props = torch.cuda.get_device_properties(local_rank)
    ident = (socket_host(), str(getattr(props, "uuid", "")) or str(local_rank),
             getattr(props, "pci_bus_id", None), local_rank)
    seen = [None] * world
    dist.all_gather_object(seen, ident)
    assert len(seen) == world, seen
    if not rehearse:
        devs = {(h, u, b) for h, u, b, _ in seen}
        if len(devs) != world:
            raise SystemExit(f"bench.py: {world} ranks share GPUs: {seen}")


def socket_host() -> str:
    import socket

    return socket.gethostname()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="roman", choices=["roman", "rmat", "arxiv", "backbone", "exact_er", "topology", "geodesic", "scorers"])
    ap.add_argument("--scale", type=int, default=22, help="R-MAT scale for --workload rmat")
    ap.add_argument("--keep", type=float, default=0.5,
                    help="--workload rmat: retention ratio of the global top-k in the step "
                         "(Jaccard-T; 1.0 = scores only)")
    ap.add_argument("--bb-graph", default="rmat", choices=["rmat", "roman"],
                    help="graph of --workload backbone (R-MAT at --bb-scale, or Roman-like)")
    ap.add_argument("--bb-scale", type=int, default=18)
    ap.add_argument("--xer-n", type=int, default=0,
                    help="--workload exact_er on a Roman-like graph of this many nodes (0: Cora size)")
    ap.add_argument("--blas-threads", type=int, default=8,
                    help="OpenBLAS ddot order to reproduce (reference run with this many threads)")
    ap.add_argument("--rng", default=os.environ.get("GSPARSE_ER_RNG", "device"),
                    choices=["host", "device"])
    ap.add_argument("--box-order-steps", type=int, default=2,
                    help="steps timed again in this box's default OpenBLAS order (secondary)")
    ap.add_argument("--cpu-sample-cols", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    rehearse = os.environ.get("GSPARSE_REHEARSE") == "1"
    if rehearse:
        # ranks sharing a GPU cannot keep every part of a split CG column resident
        os.environ.setdefault("GSPARSE_REG_SPLIT", "0")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: start the ranks before this process touches the GPU
        # (torch.cuda.device_count() does not initialise HIP on this image)
        return spawn_ranks(args.gpus, rehearse)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    visible = torch.cuda.device_count()
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if local_rank >= visible:
        if not rehearse:
            raise SystemExit(f"bench.py: LOCAL_RANK {local_rank} but only {visible} GPU(s) visible "
                             "(GSPARSE_REHEARSE=1 shares them, for rehearsals only)")
        local_rank %= max(1, visible)
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        backend = os.environ.get("GSPARSE_DIST_BACKEND", "gloo" if rehearse else "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)
        check_ranks(dist, world, local_rank, rehearse)
    dev = torch.device("cuda", local_rank)

    from gsparse import graphs
    from gsparse._lib import Context
    from gsparse.distributed import Comm, sharded_approx_er, sharded_edge_scores, sharded_sparsify
    from gsparse.engine import Engine, jl_dim

    if args.workload == "backbone":
        return bench_backbone(args, world, rank, local_rank, dev, dist)
    if args.workload == "exact_er":
        return bench_exact_er(args, world, rank, local_rank, dev, dist)
    if args.workload == "topology":
        return bench_topology(args, world, rank, local_rank, dev, dist)
    if args.workload == "geodesic":
        return bench_geodesic(args, world, rank, local_rank, dev, dist)
    if args.workload == "scorers":
        return bench_scorers(args, world, rank, local_rank, dev, dist)

    t_gen = time.perf_counter()
    if args.workload == "roman":
        ei, n = graphs.roman_like(), 22_662
        with_er = True
        wl = "configs[1] Roman-empire Jaccard+ApproxER"
    elif args.workload == "arxiv":
        ei, n = graphs.citation_like(), 169_343
        with_er = True
        wl = "configs[2] ogbn-arxiv-size Jaccard+ApproxER"
    else:
        ei, n = graphs.rmat(args.scale, 8, seed=0), 1 << args.scale
        with_er = False
        wl = f"configs[3] RMAT-{args.scale} Jaccard-T"
    t_gen = time.perf_counter() - t_gen
    E = ei.shape[1]
    ctx = Context(local_rank)
    src = torch.from_numpy(np.ascontiguousarray(ei[0])).to(dev)
    dst = torch.from_numpy(np.ascontiguousarray(ei[1])).to(dev)
    ctx.set_graph_edge_index(n, src, dst)
    del src, dst
    eng = Engine(ctx)
    nnz = eng.nnz
    k = jl_dim(n, 0.3)
    comm = Comm(device=dev) if world > 1 else None
    bounds = None  # symmetric graphs: owner-pair count shares + all-gather (sharded_jaccard)
    jac_out = torch.empty(nnz, dtype=torch.float64, device=dev)
    er_out = torch.empty(nnz, dtype=torch.float64, device=dev)

    er_cols = None
    if world > 1 and with_er:
        from gsparse.distributed import er_rank_blocks

        _, eb, runs = er_rank_blocks(k, world)
        a_, b_ = runs[rank]
        er_cols = (eb[a_], eb[b_]) if b_ > a_ else (0, 0)

    # configs[3] "Jaccard-T": the global top-k of the scores (core.py:229-240) is part of
    # the R-MAT step, on every rank after the all-gather (device tie rule)
    with_topk = args.workload == "rmat" and args.keep < 1.0
    mask_out = torch.empty(E, dtype=torch.uint8, device=dev) if with_topk else None
    sel_info = {}

    def select(scores):
        if world > 1:
            _, info = sharded_sparsify(eng, comm, scores, E, args.keep, tie_break="stable",
                                       out=mask_out)
        else:
            _, cut, nb, nt = eng.topk_mask(scores, E, int(E * args.keep), False, out=mask_out)
            info = {"cut": cut, "beyond": nb, "tied": nt}
        sel_info.update(info)

    own_scores = None
    if world > 1 and with_topk:
        from gsparse.distributed import sharded_jaccard_topk

        _, oo = eng.jaccard_shares(world)
        own_scores = torch.empty(max(1, int(oo[rank + 1] - oo[rank])), dtype=torch.float64, device=dev)

    def step():
        if world > 1 and with_topk:
            # Jaccard-T over ranks without the score exchange: own owner-pair counts and
            # scores, the cut by radix select over all-reduced histograms, one keep byte per
            # pair all-gathered, the whole mask on every rank (gs_jsel_*)
            _, info, _ = sharded_jaccard_topk(eng, comm, args.keep, tie_break="stable",
                                              mask_out=mask_out, scores_out=own_scores)
            sel_info.update(info)
            return own_scores, None
        if world > 1:
            jac = sharded_edge_scores(eng, comm, "jaccard", bounds=bounds, out=jac_out)
            er = sharded_approx_er(eng, comm, blas_threads=args.blas_threads,
                                   rng_mode=args.rng) if with_er else None
            return jac, er
        eng.jaccard(0, nnz, out=jac_out)
        if with_topk:
            select(jac_out)
        if with_er:
            rng = np.random.default_rng(42)
            eng.er_prepare(k)
            if args.rng == "device":
                eng.er_project_device(rng, k)
            else:
                eng.er_project_host(rng, k)
            eng.er_solve(0, k, 500, 1e-6, args.blas_threads)
            eng.er_scores(0, k, True, out=er_out)
        return jac_out, er_out

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.profile(True)
    ctx.profile_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = ctx.profile_read()
    ctx.profile(False)
    rank_ms = None
    if dist:
        # every rank's own time (the step time is the slowest rank's)
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if dist.get_backend() != "nccl":
            t = t.cpu()
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        rank_ms = [round(float(x.item()) * 1e3 / args.steps, 2) for x in allt]
        elapsed = max(float(x.item()) for x in allt)
    ms_per_step = elapsed * 1e3 / args.steps
    value = E * args.steps / elapsed  # every step scores all E edges (with both metrics)

    # roofline: the dominant kernel by summed time (HIP events on its stream)
    roofline = None
    if prof:
        name, p = max(((k, v) for k, v in prof.items() if v["ms"] > 0), key=lambda kv: kv[1]["ms"])
        flops = None
        if with_er and name in ("cg_reg", "cg_res"):
            # SciPy's CG does 2 nnz(L_reg) (SpMV) + 3 x 2n (dots) + 3 x 2n
            # (updates) flops per column-iteration; this rank's columns, their iterations
            c0, c1 = er_cols if er_cols else (0, k)
            its = float(eng.er_iterations()[c0:c1].astype(np.int64).sum())
            ip_h, ix_h, _ = ctx.csr()
            loops = int((np.repeat(np.arange(n), np.diff(ip_h)) == ix_h).sum())
            lnnz = nnz - loops + n  # L_reg = diag(deg) - A + 1e-6 I: every diagonal stored
            flops = (2.0 * lnnz + 12.0 * n) * its
        roofline = make_roofline(name, p["ms"] / p["launches"], p["bytes"] / p["launches"],
                                 p["launches"], args.workload, world, flops_per=flops, steps=args.steps)
    kernels = {k2: {"launches": v["launches"], "ms": round(v["ms"], 3)} for k2, v in prof.items()}

    result = {
        "metric": "scored edges/sec (Jaccard+ApproxER)" if with_er else
                  ("scored edges/sec (Jaccard-T: scores + global top-k)" if with_topk
                   else "scored edges/sec (Jaccard)"),
        "value": round(value, 1),
        "unit": "scored edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 2),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (stand-in graph of the config's size; datasets are not downloadable here)",
        "config": {"workload": wl, "n": n, "E": E, "jl_k": k if with_er else None,
                   "cg_maxiter": 500 if with_er else None,
                   "blas_threads_order": args.blas_threads, "rng": args.rng,
                   "parallelism": ((f"owner-pair shares/{world} + histogram all-reduce select"
                                    if with_topk else f"edges+jl-columns/{world}") if world > 1 else "1 GPU"),
                   "topk": ({"keep": args.keep, "num_keep": int(E * args.keep), "tie_rule": "device (stable)",
                             "tied_at_cut": sel_info.get("tied"), "beyond_cut": sel_info.get("beyond")}
                            if with_topk else None),
                   "graph_gen_s": round(t_gen, 2)},
        "roofline": roofline,
        "kernels": kernels,
    }
    if rank_ms is not None:
        result["rank_ms_per_step"] = rank_ms
    if with_topk and world == 1 and sel_info.get("tied") is not None:
        # secondary (not `value`): what the drop-in default tie_break="numpy" adds when the
        # cut is ambiguous -- the scores to the host and the reference's own np.argsort
        # (core.py:233-240) -- beside the device rule timed above
        from gsparse.selection import numpy_topk_mask

        num_keep = int(E * args.keep)
        need = num_keep - sel_info["beyond"]
        t1 = time.perf_counter()
        s_host = jac_out.cpu().numpy()
        t_d2h = time.perf_counter() - t1
        numpy_topk_mask(s_host, E, num_keep, False)
        t_sort = time.perf_counter() - t1 - t_d2h
        result["dropin_numpy_tie_break"] = {
            "ambiguous_cut": bool(0 < need < sel_info["tied"]),
            "d2h_ms": round(t_d2h * 1e3, 1), "np_argsort_mask_ms": round(t_sort * 1e3, 1),
            "step_ms_with_it": round(ms_per_step + (t_d2h + t_sort) * 1e3, 2),
            "note": "secondary: GraphSparsifier.sparsify's default tie rule resolves an ambiguous "
                    "cut with the reference's np.argsort on the host; the line's value uses the "
                    "device rule (= np.argsort(kind='stable'))"}
    if with_er and world == 1 and args.box_order_steps > 0:
        # secondary figure (not `value`): the same step in the OpenBLAS ddot order the
        # drop-in API reproduces by default on this box (threadpoolctl's thread count:
        # what the reference run here would use), beside the headline's fixed order
        from gsparse.engine import blas_threads_default

        bt_box = blas_threads_default()
        if bt_box != args.blas_threads:
            bt_main = args.blas_threads
            args.blas_threads = bt_box
            step()
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            for _ in range(args.box_order_steps):
                step()
            torch.cuda.synchronize(dev)
            ms_box = (time.perf_counter() - t1) * 1e3 / args.box_order_steps
            args.blas_threads = bt_main
        else:
            ms_box = ms_per_step
        result["box_blas_order"] = {"blas_threads": bt_box, "ms_per_step": round(ms_box, 2),
                                    "value": round(E / (ms_box * 1e-3), 1),
                                    "note": "secondary: the drop-in default order on this box"}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # one BLAS thread: the fastest setting for this SciPy CG (n=22,662) on
        # the hosts measured (8 threads: 3.8x slower from ddot threading overhead)
        if args.workload == "roman":
            result["cpu_baseline"] = cpu_baseline_roman(ei, n, args.cpu_sample_cols, 1)
        elif args.workload == "rmat":
            ip_h, ix_h, _ = ctx.csr()
            result["cpu_baseline"] = cpu_baseline_rmat(ip_h, ix_h, n, args.scale)
        elif args.workload == "arxiv":
            result["cpu_baseline"] = cpu_baseline_arxiv(ei, n)
    if rank == 0:
        emit(result)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
