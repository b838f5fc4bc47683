// gs_backbone.hip -- metric backbone prune (compute_metric_backbone,
// metric_backbone.py:28-141) on the device.
//
// Reference: G = undirected graph of the src<dst edge_index columns with
// weight min over duplicates (:70-79); APSP by Dijkstra (:86); column
// idx=(u,v) kept iff d_G(u,v) == inf or w[idx] <= d + eps (:97-111).
// Any exact SSSP whose path sums are left-folded from the source reproduces
// Dijkstra's distances bit for bit (fl(a+w) is monotone in a, so the least
// fixpoint of d(y) = min_x fl(d(x) + w(x,y)) is unique); here:
//   1. exact 2-hop witness: prune (u,v) when some common neighbour x gives
//      w_uv > fl(fl(w_ux + w_xv) + eps)  (d <= that path, so w > fl(d+eps));
//   2. for every source row u with unresolved targets: a label-correcting
//      frontier search (one workgroup per source, distances as 64-bit
//      atomicMin on the IEEE bits -- valid for non-negative doubles) pruned
//      at the largest unresolved target weight: a target beyond it has
//      d > w and is kept whatever its exact distance.
#include "gs_internal.hpp"

namespace gs {

static int bits_for_bb(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b < 1 ? 1 : b;
}

static constexpr uint64_t kInfBits = 0x7ff0000000000000ull;

__global__ void k_bb_keys(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                          const double *__restrict__ w, int64_t E, int64_t n,
                          uint64_t *__restrict__ keys, int64_t *__restrict__ idx,
                          int *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = src[i], d = dst[i];
        if (s < 0 || s >= n || d < 0 || d >= n) atomicOr(bad, 1);
        double x = w[i];
        if (!(x >= 0.0)) atomicOr(bad, 2);  // negative or NaN weight
        // undirected edges from s<d columns; others sort to the end
        keys[i] = (s < d && s >= 0 && d < n) ? (uint64_t)s * (uint64_t)n + (uint64_t)d : ~0ull;
        idx[i] = i;
    }
}

// runs of equal keys -> unique undirected edges with min weight
__global__ void k_bb_unique(const uint64_t *__restrict__ keys, const int64_t *__restrict__ idx,
                            const double *__restrict__ w, int64_t E, int64_t n,
                            unsigned long long *__restrict__ ucount, uint64_t *__restrict__ ukeys,
                            double *__restrict__ uw) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (k == ~0ull) continue;
        if (i > 0 && keys[i - 1] == k) continue;
        double m = w[idx[i]];
        for (int64_t j = i + 1; j < E && keys[j] == k; ++j) {
            double x = w[idx[j]];
            if (x < m) m = x;
        }
        if (m == 0.0) m = 0.0;
        unsigned long long p = atomicAdd(ucount, 1ull);
        uint64_t u = k / (uint64_t)n, v = k % (uint64_t)n;
        ukeys[2 * p] = u * (uint64_t)n + v;
        ukeys[2 * p + 1] = v * (uint64_t)n + u;
        uw[p] = m;
    }
}

__global__ void k_bb_sym_payload(int64_t cnt2, int64_t *__restrict__ pay) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cnt2;
         i += (int64_t)gridDim.x * blockDim.x)
        pay[i] = i >> 1;
}

__global__ void k_bb_gfill(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ pay,
                           const double *__restrict__ uw, int64_t cnt2, int64_t n,
                           int32_t *__restrict__ gi, double *__restrict__ gw,
                           unsigned long long *__restrict__ deg) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cnt2;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = skeys[i];
        gi[i] = (int32_t)(k % (uint64_t)n);
        gw[i] = uw[pay[i]];
        atomicAdd(&deg[k / (uint64_t)n], 1ull);
    }
}

__global__ void k_bb_srckeys(const int64_t *__restrict__ src, int64_t E, uint64_t *__restrict__ keys,
                             int64_t *__restrict__ idx, unsigned long long *__restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = (uint64_t)src[i];
        idx[i] = i;
        atomicAdd(&cnt[src[i]], 1ull);
    }
}

// 2-hop witness. state: 0 = unresolved, 1 = keep, 2 = prune.
__global__ void k_bb_witness(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                             const double *__restrict__ w, int64_t E,
                             const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                             const double *__restrict__ gw, double eps,
                             uint8_t *__restrict__ state) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t u = src[i], v = dst[i];
        double wi = w[i];
        if (u == v) {  // d(u,u) = 0
            state[i] = (wi <= 0.0 + eps) ? 1 : 2;
            continue;
        }
        int64_t a = gp[u], ae = gp[u + 1], b = gp[v], be = gp[v + 1];
        uint8_t st = 0;
        if (a == ae || b == be) {
            st = 1;  // u or v isolated in G: unreachable, d = inf -> keep
        } else {
            while (a < ae && b < be) {
                int32_t x = gi[a], y = gi[b];
                if (x == y) {
                    double path = gw[a] + gw[b];  // fl(fl(0 + w_ux) + w_xv)
                    if (wi > path + eps) {
                        st = 2;
                        break;
                    }
                    ++a;
                    ++b;
                } else if (x < y) {
                    ++a;
                } else {
                    ++b;
                }
            }
        }
        state[i] = st;
    }
}

// per-source bounded label-correcting search; one workgroup per source.
struct BbSlab {
    unsigned long long *dist;  // n, +inf bits when idle
    int32_t *qflag;            // n, 0 when idle
    int32_t *fa, *fb;          // frontiers, n each
    int32_t *touched;          // n
};

__global__ void __launch_bounds__(256) k_bb_sssp(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, const int64_t *__restrict__ sources, int64_t nsrc, const int64_t *__restrict__ optr,
    const int64_t *__restrict__ order, const int64_t *__restrict__ dst,
    const double *__restrict__ w, double eps, uint8_t *__restrict__ state,
    unsigned long long *__restrict__ dist_all, int32_t *__restrict__ qflag_all,
    int32_t *__restrict__ fr_all, int32_t *__restrict__ touched_all,
    unsigned long long *__restrict__ relax_total) {
    __shared__ int s_fcount, s_ncount, s_tcount;
    __shared__ double s_wmax;
    __shared__ unsigned long long s_relax;
    unsigned long long *dist = dist_all + (int64_t)blockIdx.x * n;
    int32_t *qflag = qflag_all + (int64_t)blockIdx.x * n;
    int32_t *fa = fr_all + (int64_t)blockIdx.x * 2 * n;
    int32_t *fb = fa + n;
    int32_t *touched = touched_all + (int64_t)blockIdx.x * n;
    if (threadIdx.x == 0) s_relax = 0;
    unsigned long long relax = 0;
    for (int64_t si = blockIdx.x; si < nsrc; si += gridDim.x) {
        const int64_t u = sources[si];
        const int64_t c0 = optr[u], c1 = optr[u + 1];
        if (threadIdx.x == 0) {
            s_wmax = -1.0;
            s_fcount = 1;
            s_ncount = 0;
            s_tcount = 1;
        }
        __syncthreads();
        // largest unresolved target weight
        double lm = -1.0;
        for (int64_t j = c0 + threadIdx.x; j < c1; j += blockDim.x) {
            int64_t idx = order[j];
            if (state[idx] == 0 && w[idx] > lm) lm = w[idx];
        }
        for (int off = 32; off > 0; off >>= 1) {
            double o = __shfl_down(lm, off, 64);
            lm = o > lm ? o : lm;
        }
        if ((threadIdx.x & 63) == 0) {
            // block max through a CAS loop on the bits (values >= -1)
            unsigned long long *p = (unsigned long long *)&s_wmax;
            unsigned long long old = *p;
            while (__longlong_as_double(old) < lm) {
                unsigned long long prev =
                    atomicCAS(p, old, (unsigned long long)__double_as_longlong(lm));
                if (prev == old) break;
                old = prev;
            }
        }
        __syncthreads();
        const double wmax = s_wmax;
        if (wmax < 0.0) {
            __syncthreads();
            continue;  // nothing unresolved for this source
        }
        if (threadIdx.x == 0) {
            dist[u] = 0ull;  // +0.0
            fa[0] = (int32_t)u;
            touched[0] = (int32_t)u;
        }
        __syncthreads();
        int32_t *cur = fa, *nxt = fb;
        while (true) {
            const int fc = s_fcount;
            if (fc == 0) break;
            for (int f = threadIdx.x; f < fc; f += blockDim.x) qflag[cur[f]] = 0;
            __syncthreads();
            for (int f = threadIdx.x; f < fc; f += blockDim.x) {
                const int32_t x = cur[f];
                const double dx = __longlong_as_double(
                    (long long)__hip_atomic_load(&dist[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                for (int64_t e = gp[x]; e < gp[x + 1]; ++e) {
                    ++relax;
                    const double nd = dx + gw[e];
                    if (!(nd <= wmax)) continue;
                    const int32_t y = gi[e];
                    const unsigned long long nb = (unsigned long long)__double_as_longlong(nd);
                    const unsigned long long old = atomicMin(&dist[y], nb);
                    if (nb < old) {
                        if (old == kInfBits) {
                            int t = atomicAdd(&s_tcount, 1);
                            touched[t] = y;
                        }
                        if (atomicExch(&qflag[y], 1) == 0) {
                            int q = atomicAdd(&s_ncount, 1);
                            nxt[q] = y;
                        }
                    }
                }
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                s_fcount = s_ncount;
                s_ncount = 0;
            }
            int32_t *t = cur;
            cur = nxt;
            nxt = t;
            __syncthreads();
        }
        // classify unresolved targets
        for (int64_t j = c0 + threadIdx.x; j < c1; j += blockDim.x) {
            int64_t idx = order[j];
            if (state[idx] != 0) continue;
            int64_t v = dst[idx];
            unsigned long long db =
                __hip_atomic_load(&dist[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            double d = __longlong_as_double((long long)db);
            bool keep = (db == kInfBits) || (w[idx] <= d + eps);
            state[idx] = keep ? 1 : 2;
        }
        __syncthreads();
        const int tc = s_tcount;
        for (int t = threadIdx.x; t < tc; t += blockDim.x) {
            int32_t y = touched[t];
            dist[y] = kInfBits;
            qflag[y] = 0;
        }
        __syncthreads();
    }
    atomicAdd(&s_relax, relax);
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(relax_total, s_relax);
}

__global__ void k_bb_fill_u64(unsigned long long *p, int64_t n, unsigned long long v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// sources: rows with at least one unresolved target
__global__ void k_bb_need(const int64_t *__restrict__ optr, const int64_t *__restrict__ order,
                          const uint8_t *__restrict__ state, int64_t n, int64_t *__restrict__ flag) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        int64_t f = 0;
        for (int64_t j = optr[u]; j < optr[u + 1]; ++j)
            if (state[order[j]] == 0) {
                f = 1;
                break;
            }
        flag[u] = f;
    }
}

__global__ void k_bb_compact(const int64_t *__restrict__ flag, const int64_t *__restrict__ pos,
                             int64_t n, int64_t *__restrict__ sources) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x)
        if (flag[u]) sources[pos[u]] = u;
}

__global__ void k_bb_keep(const uint8_t *__restrict__ state, int64_t E, uint8_t *__restrict__ keep) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        keep[i] = state[i] == 1;
}

}  // namespace gs

using namespace gs;

extern "C" int gs_metric_backbone(gs_ctx *c, int64_t n, int64_t E, const int64_t *src,
                                  const int64_t *dst, const double *w, int loc, double eps,
                                  uint8_t *keep, int keep_loc, int64_t *n_relax) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(n >= 0 && E >= 0, GS_EINVAL, "negative n/E");
        GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        // own buffers (the scorer scratch slots stay untouched)
#define BB(name) DevBuf &b_##name = c->buf("bb_" #name)
        BB(src); BB(dst); BB(w); BB(keys); BB(idx); BB(ukeys); BB(uw); BB(pay); BB(gp); BB(gi);
        BB(gw); BB(okeys); BB(order); BB(optr); BB(state); BB(flag); BB(pos); BB(sources);
        BB(dist); BB(qflag); BB(fr); BB(touched); BB(misc); BB(keep);
#undef BB
        const int64_t *dsrc =
            (const int64_t *)to_device(c, b_src, src, sizeof(int64_t) * E, loc);
        const int64_t *ddst =
            (const int64_t *)to_device(c, b_dst, dst, sizeof(int64_t) * E, loc);
        const double *dw = (const double *)to_device(c, b_w, w, sizeof(double) * E, loc);
        uint8_t *dkeep = (uint8_t *)out_device(c, b_keep, keep, E ? E : 1, keep_loc);
        unsigned long long *misc = (unsigned long long *)b_misc.ensure(64);
        GS_HIP(hipMemsetAsync(misc, 0, 64, s));
        int64_t relax = 0;
        hipEvent_t t0 = prof_begin(c);
        if (E > 0) {
            int *bad = (int *)(misc + 4);
            uint64_t *keys = (uint64_t *)b_keys.ensure(8 * E);
            int64_t *idx = (int64_t *)b_idx.ensure(8 * E);
            k_bb_keys<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, ddst, dw, E, n, keys, idx, bad);
            int hbad = 0;
            GS_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            GS_CHECK(!(hbad & 1), GS_EINVAL, "edge_index entry out of range [0, %lld)", (long long)n);
            GS_CHECK(!(hbad & 2), GS_EUNSUPPORTED,
                     "edge weights must be non-negative and not NaN (Dijkstra contract)");
            sort_pairs_u64_i64(c, keys, idx, E, 64);
            uint64_t *ukeys = (uint64_t *)b_ukeys.ensure(16 * E);
            double *uw = (double *)b_uw.ensure(8 * E);
            k_bb_unique<<<grid_for(E, 256, 8192), 256, 0, s>>>(keys, idx, dw, E, n, misc, ukeys, uw);
            unsigned long long ucnt = 0;
            GS_HIP(hipMemcpyAsync(&ucnt, misc, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            int64_t cnt2 = 2 * (int64_t)ucnt;
            // G as symmetric CSR sorted by (row, col): unique keys -> no ties in order
            int64_t *pay = (int64_t *)b_pay.ensure(8 * (cnt2 + 1));
            k_bb_sym_payload<<<grid_for(cnt2 + 1, 256, 8192), 256, 0, s>>>(cnt2, pay);
            sort_pairs_u64_i64(c, ukeys, pay, cnt2, bits_for_bb((uint64_t)n * (uint64_t)n));
            int64_t *gp = (int64_t *)b_gp.ensure(8 * (n + 1));
            int32_t *gi = (int32_t *)b_gi.ensure(4 * (cnt2 + 1));
            double *gw = (double *)b_gw.ensure(8 * (cnt2 + 1));
            unsigned long long *deg = (unsigned long long *)b_flag.ensure(8 * (n + 1));
            GS_HIP(hipMemsetAsync(deg, 0, 8 * (n + 1), s));
            if (cnt2)
                k_bb_gfill<<<grid_for(cnt2, 256, 8192), 256, 0, s>>>(ukeys, pay, uw, cnt2, n, gi, gw,
                                                                    deg);
            exclusive_scan_i64(c, (const int64_t *)deg, gp, n + 1);
            // columns grouped by source row (stable: radix sort is stable)
            uint64_t *okeys = (uint64_t *)b_okeys.ensure(8 * E);
            int64_t *order = (int64_t *)b_order.ensure(8 * E);
            int64_t *optr = (int64_t *)b_optr.ensure(8 * (n + 1));
            GS_HIP(hipMemsetAsync(deg, 0, 8 * (n + 1), s));
            k_bb_srckeys<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, E, okeys, order, deg);
            sort_pairs_u64_i64(c, okeys, order, E, bits_for_bb((uint64_t)n));
            exclusive_scan_i64(c, (const int64_t *)deg, optr, n + 1);
            // 2-hop witness
            uint8_t *state = (uint8_t *)b_state.ensure(E);
            k_bb_witness<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, ddst, dw, E, gp, gi, gw, eps,
                                                               state);
            // sources needing a search
            int64_t *flag = (int64_t *)b_flag.ensure(8 * (n + 1));
            int64_t *pos = (int64_t *)b_pos.ensure(8 * (n + 1));
            k_bb_need<<<grid_for(n, 256, 8192), 256, 0, s>>>(optr, order, state, n, flag);
            exclusive_scan_i64(c, flag, pos, n);
            int64_t lastp = 0, lastf = 0;
            if (n) {
                GS_HIP(hipMemcpyAsync(&lastp, pos + n - 1, 8, hipMemcpyDeviceToHost, s));
                GS_HIP(hipMemcpyAsync(&lastf, flag + n - 1, 8, hipMemcpyDeviceToHost, s));
            }
            GS_HIP(hipStreamSynchronize(s));
            int64_t nsrc = lastp + lastf;
            if (nsrc > 0) {
                int64_t *sources = (int64_t *)b_sources.ensure(8 * nsrc);
                k_bb_compact<<<grid_for(n, 256, 8192), 256, 0, s>>>(flag, pos, n, sources);
                int64_t slabs = nsrc < 1024 ? nsrc : 1024;
                // keep the per-slab working set under ~8 GB
                int64_t cap = (int64_t)(8e9 / (24.0 * (double)(n ? n : 1)));
                if (cap < 1) cap = 1;
                if (slabs > cap) slabs = cap;
                unsigned long long *dist = (unsigned long long *)b_dist.ensure(8 * slabs * n);
                int32_t *qflag = (int32_t *)b_qflag.ensure(4 * slabs * n);
                int32_t *fr = (int32_t *)b_fr.ensure(8 * slabs * n);
                int32_t *touched = (int32_t *)b_touched.ensure(4 * slabs * n);
                k_bb_fill_u64<<<grid_for(slabs * n, 256, 65536), 256, 0, s>>>(dist, slabs * n,
                                                                               kInfBits);
                GS_HIP(hipMemsetAsync(qflag, 0, 4 * slabs * n, s));
                k_bb_sssp<<<(unsigned)slabs, 256, 0, s>>>(gp, gi, gw, n, sources, nsrc, optr, order,
                                                          ddst, dw, eps, state, dist, qflag, fr,
                                                          touched, misc + 1);
                GS_HIP(hipGetLastError());
            }
            k_bb_keep<<<grid_for(E, 256, 8192), 256, 0, s>>>(state, E, dkeep);
            unsigned long long hr = 0;
            GS_HIP(hipMemcpyAsync(&hr, misc + 1, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            relax = (int64_t)hr;
        }
        prof_end(c, t0, "metric_backbone", 12.0 * (double)relax + 9.0 * (double)E);
        finish_out(c, keep, dkeep, E, keep_loc);
        if (n_relax) *n_relax = relax;
    });
}
