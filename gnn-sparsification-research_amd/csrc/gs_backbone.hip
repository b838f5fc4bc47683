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

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace gs {

static int bits_for_bb(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b < 1 ? 1 : b;
}

static constexpr uint64_t kInfBits = 0x7ff0000000000000ull;
static constexpr int kBbLandmarkRounds = 256;  // frontier rounds per landmark search
// k_bb_sssp_multi's per-node mask: bits 0-7 the sources queued in the next frontier,
// 8-15 the sources for which the node waits in the far pile, 30 the node is in the
// far list, 31 in the reset list
static constexpr uint32_t kQMaskTouched = 0x80000000u;
static constexpr uint32_t kQMaskFarListed = 0x40000000u;
static constexpr uint32_t kQMaskSources = 0xffu;
static constexpr int kQMaskFarShift = 8;
// k_bb_sssp_multi: frontier nodes with more entries than this are expanded by the
// whole workgroup (at most kBbHeavyMax of them per round; the rest as usual)
#ifndef GS_BB_HEAVY
#define GS_BB_HEAVY 1024
#endif
static constexpr int64_t kBbHeavy = GS_BB_HEAVY;
static constexpr int kBbHeavyMax = 256;

// Which rule decided a column (gs_bb_classes / gs_bb_class_counts; include/gsparse.h
// GS_BB_WHY_*).  Recorded only when the caller asks (why != null): a diagnostic for the
// parity tests, which assert that every certificate class fires on their graphs.
enum : uint8_t {
    kWhyOpen = 0,      // not decided by this rank
    kWhySelf,          // self-loop: d(u, u) = 0
    kWhyIsolated,      // an endpoint without G edges: d = inf, keep
    kWhyDeg1,          // an endpoint of degree 1 whose only neighbour is the other: d = w_G
    kWhyDirect,        // w > fl(w_G + eps): prune
    kWhyLocal2,        // w <= fl(mu' + mv')(1 - 2m): keep
    kWhyLmComp,        // a complete landmark reaches one endpoint only: keep
    kWhyLmPrune,       // landmark upper bound: prune
    kWhyLmKeep,        // landmark lower bound: keep
    kWhyWitness,       // 2-hop path: prune
    kWhyLocal34,       // 2- / 3- / 4-edge local lower bound: keep
    kWhySearchPrune,   // the row's search: prune
    kWhySearchKeep,    // the row's search: keep
    kWhyRevExact,      // the reverse row's search, exact rule
    kWhyRevPrune,      // the reverse row's search, upper bound: prune
    kWhyRevKeep,       // the reverse row's search, v unreached within the bound: keep
    kWhyMitm,          // meet-in-the-middle certificate (GSPARSE_BB_MITM)
    kWhyClasses
};
__device__ __forceinline__ void bb_set(uint8_t *__restrict__ state, uint8_t *__restrict__ why, int64_t i,
                                       uint8_t st, uint8_t cls) {
    state[i] = st;
    if (why) why[i] = cls;
}

// osrc/odst: the caller's ids (which columns are s < d: metric_backbone.py:70-79
// builds G from those); src/dst: the (possibly relabeled) ids G is built in
__global__ void k_bb_keys(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                          const int64_t *__restrict__ osrc, const int64_t *__restrict__ odst,
                          const double *__restrict__ w, int64_t E, int64_t n,
                          uint64_t *__restrict__ keys, int64_t *__restrict__ idx,
                          int *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t os = osrc[i], od = odst[i];
        if (os < 0 || os >= n || od < 0 || od >= n) {
            atomicOr(bad, 1);
            keys[i] = (uint64_t)n * (uint64_t)n;
            idx[i] = i;
            continue;
        }
        const int64_t s = src[i], d = dst[i];
        double x = w[i];
        if (!(x >= 0.0)) atomicOr(bad, 2);  // negative or NaN weight
        // undirected edges from s<d columns (caller's ids); others sort to the end
        const uint64_t lo = (uint64_t)(s < d ? s : d), hi = (uint64_t)(s < d ? d : s);
        keys[i] = os < od ? lo * (uint64_t)n + hi : (uint64_t)n * (uint64_t)n;
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
        if (k >= (uint64_t)n * (uint64_t)n) continue;
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
                           int32_t *__restrict__ gi, double *__restrict__ gw) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cnt2;
         i += (int64_t)gridDim.x * blockDim.x) {
        gi[i] = (int32_t)(skeys[i] % (uint64_t)n);
        gw[i] = uw[pay[i]];
    }
}

// row pointers of keys sorted by row = key / div (rows < n): ptr[r] = the first entry whose
// key is >= r * div, one binary search per row (no atomics: an R-MAT hub's degree counted
// by atomics on one address serialises -- the G fill and the columns-by-row pass took
// 1.6 + 1.2 ms of RMAT-18's begin, round 5; and no per-entry loop over the empty rows
// between entries: the degree relabeling puts ~40 % of the rows, all empty, last)
__global__ void k_bb_rowptr(const uint64_t *__restrict__ keys, int64_t cnt, uint64_t div, int64_t n,
                            int64_t *__restrict__ ptr) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= n;
         r += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t t = (uint64_t)r * div;
        int64_t lo = 0, hi = cnt;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (keys[mid] < t) lo = mid + 1;
            else hi = mid;
        }
        ptr[r] = lo;
    }
}

__global__ void k_bb_srckeys(const int64_t *__restrict__ src, int64_t E, uint64_t *__restrict__ keys,
                             int64_t *__restrict__ idx) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = (uint64_t)src[i];
        idx[i] = i;
    }
}

// Part of a column in the sharded form: both columns (u, v) and (v, u) of a pair go to
// the part of its lower-degree endpoint (the larger id after the relabeling, the
// caller's larger id without it), so one part decides both directions of a pair and
// a search's reverse-column decisions (bb_cross_decide) stay within the part.
__device__ __forceinline__ int bb_col_part(int64_t u, int64_t v, int nparts) {
    return (int)((u > v ? u : v) % nparts);
}

// 2-hop witness. state: 0 = unresolved, 1 = keep, 2 = prune.
// Columns [c0, c1) only (the staged multi-rank form splits them in ranges; the rest
// keep their state).  Pair form (nparts > 1): only the columns of this part
// (bb_col_part) are decided here: the other parts' columns are marked 3 and never
// decided by this part (k_bb_need, k_bb_keep).
// With the local bounds (mw != null; k_bb_certify has pruned every column heavier than
// its own G edge + eps): a column the 2-hop paths do not prune is kept when
// w <= LB (1 - 2m), LB = min(W2, max(Au' + mv', mu' + Av'), Au' + Av') -- W2 the least
// 2-edge fold (+inf: no common neighbour), mu' / mv' the least other edge weights of
// u / v, Au' = min over u's other neighbours a of w_ua + (a's least edge weight but
// (a, u)) (k_bb_minw2): a 3-edge path u-a-b-v is at least Au' + w_bv >= Au' + mv' and
// at least mu' + Av'; a longer one's first two and last two edges are distinct,
// >= Au' + Av'.  (R-MAT-15: 93.5 % of the kept columns certified, 66 % by mu' + mv'.)
__global__ void k_bb_witness(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                             const double *__restrict__ w, int64_t c0, int64_t c1,
                             const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                             const double *__restrict__ gw, double eps, int part, int nparts,
                             const double *__restrict__ mw, const int32_t *__restrict__ ma,
                             const double *__restrict__ aw, const int32_t *__restrict__ aa,
                             double m, uint8_t *__restrict__ state, uint8_t *__restrict__ why) {
    for (int64_t i = c0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c1;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t u = src[i], v = dst[i];
        if (nparts > 1 && bb_col_part(u, v, nparts) != part) {
            state[i] = 3;  // another part's column: not decided here
            continue;
        }
        if (state[i] != 0) continue;  // decided by k_bb_certify (it runs first)
        double wi = w[i];
        if (u == v) {  // d(u,u) = 0
            bb_set(state, why, i, (wi <= 0.0 + eps) ? 1 : 2, kWhySelf);
            continue;
        }
        int64_t a = gp[u], ae = gp[u + 1], b = gp[v], be = gp[v + 1];
        uint8_t st = 0, cls = kWhyOpen;
        double w2 = __builtin_inf();
        if (a == ae || b == be) {
            st = 1;  // u or v isolated in G: unreachable, d = inf -> keep
            cls = kWhyIsolated;
        } else {
            while (a < ae && b < be) {
                int32_t x = gi[a], y = gi[b];
                if (x == y) {
                    double path = gw[a] + gw[b];  // fl(fl(0 + w_ux) + w_xv)
                    if (wi > path + eps) {
                        st = 2;
                        cls = kWhyWitness;
                        break;
                    }
                    w2 = path < w2 ? path : w2;
                    ++a;
                    ++b;
                } else if (x < y) {
                    ++a;
                } else {
                    ++b;
                }
            }
            if (st == 0 && aw) {
                const double mu = ma[u] == (int32_t)v ? mw[2 * u + 1] : mw[2 * u];
                const double mv = ma[v] == (int32_t)u ? mw[2 * v + 1] : mw[2 * v];
                const double au = aa[u] == (int32_t)v ? aw[2 * u + 1] : aw[2 * u];
                const double av = aa[v] == (int32_t)u ? aw[2 * v + 1] : aw[2 * v];
                const double l3a = au + mv, l3b = mu + av, l3 = l3a > l3b ? l3a : l3b, l4 = au + av;
                double lb = w2 < l3 ? w2 : l3;
                lb = lb < l4 ? lb : l4;
                if (wi <= lb * (1.0 - 2.0 * m)) {
                    st = 1;
                    cls = kWhyLocal34;
                }
            }
        }
        state[i] = st;
        if (why && st) why[i] = cls;
    }
}

// per-source bounded label-correcting search; one workgroup per source.
struct BbSlab {
    unsigned long long *dist;  // n, +inf bits when idle
    int32_t *qflag;            // n, 0 when idle
    int32_t *fa, *fb;          // frontiers, n each
    int32_t *touched;          // n
};

// Bounded label-correcting search from u over G: dist[] (IEEE bits, +inf when
// idle) holds the least fixpoint of d(y) = min_x fl(d(x) + w(x,y)) restricted
// to values <= the bound s_wmax; touched[0 .. s_tcount) lists every node it
// wrote.  After every frontier round the whole workgroup runs hook(), which
// may lower s_wmax (never below a distance still needed) or end the search by
// zeroing s_fcount; a node whose true distance is <= the final bound gets its
// exact value, since no relaxation on its shortest path was ever cut.
template <class Hook>
__device__ void bb_search(const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                          const double *__restrict__ gw, int32_t u, const double &s_wmax,
                          unsigned long long *__restrict__ dist, int32_t *__restrict__ qflag,
                          int32_t *__restrict__ fa, int32_t *__restrict__ fb,
                          int32_t *__restrict__ touched, int &s_fcount, int &s_ncount,
                          int &s_tcount, unsigned long long &relax, Hook hook) {
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
        const double wmax = s_wmax;
        for (int f = threadIdx.x; f < fc; f += blockDim.x) qflag[cur[f]] = 0;
        __syncthreads();
        // edge-parallel expansion: each wave takes 64 frontier nodes, scans their
        // degrees, and its lanes walk the concatenated edge lists 64 at a time
        // (coalesced, balanced across hubs and leaves); a relaxation only
        // issues the 64-bit atomicMin after a plain load shows it improves
        __shared__ int32_t w_pre[16][65];  // per wave (blocks of up to 1024 threads)
        __shared__ int64_t w_beg[16][64];
        __shared__ double w_d[16][64];
        const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
        for (int f0 = wv * 64; f0 < fc; f0 += (int)blockDim.x) {
            const int f = f0 + lane;
            int deg = 0;
            int64_t b = 0;
            double dx = 0.0;
            if (f < fc) {
                const int32_t x = cur[f];
                b = gp[x];
                deg = (int)(gp[x + 1] - b);
                dx = __longlong_as_double(
                    (long long)__hip_atomic_load(&dist[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            }
            int incl = deg;
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            const int total = __shfl(incl, 63, 64);
            w_pre[wv][lane + 1] = incl;
            if (lane == 0) w_pre[wv][0] = 0;
            w_beg[wv][lane] = b;
            w_d[wv][lane] = dx;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            constexpr int U = 4;  // edges per lane per trip, all loads in flight
            for (int e0 = 0; e0 < total; e0 += 64 * U) {
                int32_t y[U];
                unsigned long long nb[U], cur_d[U];
                bool go[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int e = e0 + u * 64 + lane;
                    go[u] = e < total;
                    const int ec = go[u] ? e : 0;
                    int lo = 0, hi = 63;  // largest k with w_pre[k] <= ec
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (w_pre[wv][mid] <= ec) lo = mid;
                        else hi = mid - 1;
                    }
                    const int64_t ei = w_beg[wv][lo] + (ec - w_pre[wv][lo]);
                    relax += go[u] ? 1 : 0;
                    const double nd = w_d[wv][lo] + gw[ei];
                    go[u] = go[u] && (nd <= wmax);
                    y[u] = gi[ei];
                    nb[u] = (unsigned long long)__double_as_longlong(nd);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    cur_d[u] = go[u] ? __hip_atomic_load(&dist[y[u]], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP)
                                     : 0ull;
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (!go[u] || nb[u] >= cur_d[u]) continue;
                    const unsigned long long old = atomicMin(&dist[y[u]], nb[u]);
                    if (nb[u] < old) {
                        if (old == kInfBits) {
                            int t = atomicAdd(&s_tcount, 1);
                            touched[t] = y[u];
                        }
                        if (atomicExch(&qflag[y[u]], 1) == 0) {
                            int q = atomicAdd(&s_ncount, 1);
                            nxt[q] = y[u];
                        }
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
        hook();
    }
}

// block-wide max of v (values >= -1) into *out, which holds -1 on entry;
// ends with a barrier
__device__ void bb_block_max(double v, double *out) {
    for (int off = 32; off > 0; off >>= 1) {
        double o = __shfl_down(v, off, 64);
        v = o > v ? o : v;
    }
    if ((threadIdx.x & 63) == 0) {
        unsigned long long *p = (unsigned long long *)out;
        unsigned long long old = *p;
        while (__longlong_as_double(old) < v) {
            unsigned long long prev = atomicCAS(p, old, (unsigned long long)__double_as_longlong(v));
            if (prev == old) break;
            old = prev;
        }
    }
    __syncthreads();
}

template <int NT>
__global__ void __launch_bounds__(NT) k_bb_sssp(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, const int64_t *__restrict__ sources, int64_t nsrc, const int64_t *__restrict__ optr,
    const int64_t *__restrict__ order, const int64_t *__restrict__ dst,
    const double *__restrict__ w, double eps, uint8_t *__restrict__ state,
    unsigned long long *__restrict__ dist_all, int32_t *__restrict__ qflag_all,
    int32_t *__restrict__ fr_all, int32_t *__restrict__ touched_all, int64_t b0, int64_t b1,
    int part, int nparts, unsigned long long *__restrict__ relax_total, uint8_t *__restrict__ why) {
    __shared__ int s_fcount, s_ncount, s_tcount;
    __shared__ double s_wmax, s_wnext;
    __shared__ unsigned long long s_relax;
    unsigned long long *dist = dist_all + (int64_t)blockIdx.x * n;
    int32_t *qflag = qflag_all + (int64_t)blockIdx.x * n;
    int32_t *fa = fr_all + (int64_t)blockIdx.x * 2 * n;
    int32_t *fb = fa + n;
    int32_t *touched = touched_all + (int64_t)blockIdx.x * n;
    if (threadIdx.x == 0) s_relax = 0;
    unsigned long long relax = 0;
    // sources [b0, b1) of the list (b1 <= nsrc), this part's every nparts-th one
    for (int64_t j = blockIdx.x;; j += gridDim.x) {
        const int64_t si = b0 + part + j * nparts;
        if (si >= b1) break;
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
        bb_block_max(lm, &s_wmax);
        if (s_wmax < 0.0) {
            __syncthreads();
            continue;  // nothing unresolved for this source
        }
        // after each round: a target whose current (upper-bound) distance
        // already proves w > fl(d + eps) is pruned for good; the bound drops to
        // the largest weight still undecided, and the search ends when none is
        auto hook = [&]() {
            if (threadIdx.x == 0) s_wnext = -1.0;
            __syncthreads();
            double m = -1.0;
            for (int64_t j = c0 + threadIdx.x; j < c1; j += blockDim.x) {
                const int64_t idx = order[j];
                if (state[idx] != 0) continue;
                const unsigned long long db =
                    __hip_atomic_load(&dist[dst[idx]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (db != kInfBits && w[idx] > __longlong_as_double((long long)db) + eps) {
                    bb_set(state, why, idx, 2, kWhySearchPrune);
                    continue;
                }
                m = w[idx] > m ? w[idx] : m;
            }
            bb_block_max(m, &s_wnext);
            if (threadIdx.x == 0) {
                s_wmax = s_wnext;
                if (s_wnext < 0.0) s_fcount = 0;
            }
            __syncthreads();
        };
        bb_search(gp, gi, gw, (int32_t)u, s_wmax, dist, qflag, fa, fb, touched, s_fcount,
                  s_ncount, s_tcount, relax, hook);
        // classify unresolved targets
        for (int64_t j = c0 + threadIdx.x; j < c1; j += blockDim.x) {
            int64_t idx = order[j];
            if (state[idx] != 0) continue;
            int64_t v = dst[idx];
            unsigned long long db =
                __hip_atomic_load(&dist[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            double d = __longlong_as_double((long long)db);
            bool keep = (db == kInfBits) || (w[idx] <= d + eps);
            bb_set(state, why, idx, keep ? 1 : 2, keep ? kWhySearchKeep : kWhySearchPrune);
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

// Lower a label whose prefetched value was above nb.  GS_BB_NORET: fire and forget
// (the wave does not wait for the atomic's return), and y counts as improved on the
// prefetched value alone -- when another lane got there first, y is queued for a
// source whose label it did not lower, an extra expansion that changes no fixpoint.
#ifndef GS_BB_NORET
#define GS_BB_NORET 1
#endif
__device__ __forceinline__ bool bb_min_improves(unsigned long long *p, unsigned long long nb) {
#if GS_BB_NORET
    atomicMin(p, nb);
    return true;
#else
    return nb < atomicMin(p, nb);
#endif
}

// Reverse columns (metric_backbone.py:97-111 decides column (v, u) from v's Dijkstra,
// column (u, v) from u's).  After u's search, D = u's label of v (the left fold of a
// real u-v path; m bounds the relative rounding of folds over simple paths, as in
// k_bb_certify):
//  * prune: d_fl(v, u) <= D (1 + m) (the same path folded from v), so a reverse
//    column with w > (D (1 + m) + eps)(1 + m) is pruned;
//  * exact: when u's search ran dry within bound bk >= D (frontier empty), labels
//    <= bk are exact and every other label exceeds bk, so A = min over v's other G
//    neighbours x of (label(x), or bk if beyond it) + w(x, v) bounds every u-v path
//    but the edge itself from below: real length >= A (1 - m).  A (1 - 3m) > D then
//    means the edge is the only shortest path from either end by more than any
//    rounding, so d_fl(v, u) = fl(0 + w_G) = D exactly, and the reverse column is
//    decided as the reference decides it: w <= D + eps.  (A v of more than
//    kBbCrossDeg neighbours -- a hub the search reached -- is scanned by the whole
//    workgroup after the classification, up to kBbCrossBig of them per batch.)
//  * keep, v unreached: d_fl(u, v) > bk, so w <= (bk (1 - m) + eps)(1 - m) keeps it.
// Whatever falls within the margins stays open for v's own search.
// skeys / sidx: every column's (row * n + col) key in ascending order and its column;
// rp: the first position of the reverse key (-1: none).
#ifndef GS_BB_CROSS_DEG
#define GS_BB_CROSS_DEG 128
#endif
static constexpr int64_t kBbCrossDeg = GS_BB_CROSS_DEG;
#ifndef GS_BB_CROSS_BIG
#define GS_BB_CROSS_BIG 1024
#endif
static constexpr int kBbCrossBig = GS_BB_CROSS_BIG;
template <int S>
__device__ __forceinline__ bool bb_cross_decide(const uint64_t *__restrict__ skeys,
                                                const int64_t *__restrict__ sidx, int64_t rp,
                                                int64_t u, int64_t v, int64_t n, int64_t E,
                                                int k, unsigned long long db, double bk, double m,
                                                double eps, const double *__restrict__ w,
                                                const int64_t *__restrict__ gp,
                                                const int32_t *__restrict__ gi,
                                                const double *__restrict__ gw,
                                                const unsigned long long *__restrict__ dist,
                                                uint8_t *__restrict__ state, uint8_t *__restrict__ why) {
    if (rp < 0) return false;
    const uint64_t rkey = (uint64_t)v * (uint64_t)n + (uint64_t)u;
    bool open = false;  // any reverse column still undecided
    for (int64_t p = rp; p < E && skeys[p] == rkey; ++p) open = open || state[sidx[p]] == 0;
    if (!open) return false;
    const bool reached = db != kInfBits;
    const double D = __longlong_as_double((long long)db);
    bool exact = false;
    const bool eligible = reached && bk >= 0.0 && D <= bk;
    if (eligible && gp[v + 1] - gp[v] <= kBbCrossDeg) {
        double A = __longlong_as_double((long long)kInfBits);
        for (int64_t e = gp[v]; e < gp[v + 1]; ++e) {
            const int32_t x = gi[e];
            if (x == u) continue;
            const unsigned long long bx = __hip_atomic_load(&dist[(int64_t)x * S + k], __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP);
            const double dx = __longlong_as_double((long long)bx);
            const double lb = (bx != kInfBits && dx <= bk) ? dx : bk;
            const double a = lb + gw[e];
            A = a < A ? a : A;
        }
        exact = A * (1.0 - 3.0 * m) > D;
    }
    const double hi = reached ? (D * (1.0 + m) + eps) * (1.0 + m) : 0.0;
    const bool keep_unreached = !reached && bk >= 0.0;
    const double lo = keep_unreached ? (bk * (1.0 - m) + eps) * (1.0 - m) : -1.0;
    bool left = false;
    for (int64_t p = rp; p < E && skeys[p] == rkey; ++p) {
        const int64_t r = sidx[p];
        if (state[r] != 0) continue;
        const double wr = w[r];
        if (exact) bb_set(state, why, r, wr <= D + eps ? 1 : 2, kWhyRevExact);
        else if (reached && wr > hi) bb_set(state, why, r, 2, kWhyRevPrune);
        else if (keep_unreached && wr <= lo) bb_set(state, why, r, 1, kWhyRevKeep);
        else left = true;
    }
    // a v of more than kBbCrossDeg neighbours: the caller's workgroup scans them
    return left && eligible && gp[v + 1] - gp[v] > kBbCrossDeg;
}

// (row * n + col) key of every column, for the reverse-column lookup
__global__ void k_bb_pairkeys(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                              int64_t E, int64_t n, uint64_t *__restrict__ keys,
                              int64_t *__restrict__ idx) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        keys[i] = (uint64_t)src[i] * (uint64_t)n + (uint64_t)dst[i];
        idx[i] = i;
    }
}

// first position of column i's reverse key (col * n + row) in the sorted keys, -1 if
// absent or a self-loop
__global__ void k_bb_revpos(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                            int64_t E, int64_t n, const uint64_t *__restrict__ skeys,
                            int64_t *__restrict__ rpos) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[i], v = dst[i];
        const uint64_t key = (uint64_t)v * (uint64_t)n + (uint64_t)u;
        int64_t lo = 0, hi = E;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (skeys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        rpos[i] = (u != v && lo < E && skeys[lo] == key) ? lo : -1;
    }
}

// order-preserving u64 key of a double (0 below every key: "no value")
__device__ __forceinline__ unsigned long long dkey(double v) {
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double dkey_val(unsigned long long k) {
    return __longlong_as_double((long long)((k >> 63) ? (k & 0x7fffffffffffffffull) : ~k));
}

// S per-source maxima at once: each thread's keys -> wave max -> one LDS atomicMax
// per wave and source into out[S] (0 on entry); ends with a barrier
template <int S>
__device__ __forceinline__ void bb_block_max_s(unsigned long long (&m)[S], unsigned long long *out) {
#pragma unroll
    for (int k = 0; k < S; ++k) {
        unsigned long long v = m[k];
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(v, off, 64);
            v = o > v ? o : v;
        }
        if ((threadIdx.x & 63) == 0 && v) atomicMax(&out[k], v);
    }
    __syncthreads();
}

// S sources per workgroup, searched together: dist[x*S + s] interleaved, so
// the random read of node x's labels is one 8S-byte segment shared by the S
// searches (the single-source kernel fetches a whole line per relaxation).
// The frontier is the union of the sources' frontiers; qmask[x] holds the
// sources whose label of x improved in the round (x is queued once).  Each
// source keeps its own bound s_wmax[s], lowered by its own targets exactly as
// in k_bb_sssp, so every source reaches the same fixpoint as alone.
// Near-far order (delta > 0): an improvement to a label >= the source's
// threshold s_thr[s] waits in the far pile instead of the next frontier; when
// a source has nothing near left its threshold moves to (least pending far
// label) + delta and the far labels below it join the frontier.  Labels are
// then mostly expanded once at their final value (a plain frontier search
// re-expands ~1.9x as many on RMAT-18's Jaccard costs; near-far ~1.05x at
// delta = median weight / 2, tools/bb_nearfar_sim.c) -- the fixpoint, and so
// every distance and decision, is the same in any order.
// PAIR (S = 2; the meet-in-the-middle certificate, bb_pair_certify): batch b searches
// both ends of the open column sources[b] = i (src[i], dst[i]) to the radius
// r = w_max (1 + 8m) / 2, w_max the larger of its and its reverse columns' weights, with
// no target pruning, then decides the column and its reverse columns where the balls
// prove it (see the evaluation below).
template <int NT, int S, bool PAIR = false>
__global__ void __launch_bounds__(NT) k_bb_sssp_multi(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, const int64_t *__restrict__ sources, int64_t nsrc, const int64_t *__restrict__ optr,
    const int64_t *__restrict__ order, const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
    const double *__restrict__ w, double eps, uint8_t *__restrict__ state,
    unsigned long long *__restrict__ dist_all, uint32_t *__restrict__ qmask_all,
    int32_t *__restrict__ fr_all, uint32_t *__restrict__ fm_all, int32_t *__restrict__ touched_all,
    int32_t *__restrict__ far_all, double delta, int cross, const uint64_t *__restrict__ skeys,
    const int64_t *__restrict__ sidx, const int64_t *__restrict__ rpos, int64_t E, double mrg,
    int rev, int64_t b0, int64_t b1, int part, int nparts,
    unsigned long long *__restrict__ batch_next, unsigned long long *__restrict__ relax_total,
    unsigned long long *__restrict__ trace, uint8_t *__restrict__ why,
    const uint8_t *__restrict__ lmflag = nullptr, const double *__restrict__ LD = nullptr,
    const int32_t *__restrict__ lcomp = nullptr, int K = 0) {
    static_assert(S >= 1 && S <= 16, "1..16 sources per workgroup");
    static_assert(!PAIR || S == 2, "the pair form searches both ends of one column");
    // queue bits of the per-node mask; the near-far order needs S more bits for the
    // far pile (S <= 8 only: 16 sources fill the word)
    constexpr uint32_t QS = S <= 8 ? kQMaskSources : 0xffffu;
    constexpr bool NF = S <= 8;
    if (!NF) delta = 0.0;
    constexpr int NW = NT / 64;
    __shared__ int s_fcount, s_ncount, s_tcount, s_nfar, s_nfar2, s_farleft, s_nheavy, s_nbig;
    __shared__ int64_t s_big[kBbCrossBig];  // deferred reverse decisions: idx << 4 | source k
    __shared__ unsigned long long s_amin;
    __shared__ int32_t s_heavy[kBbHeavyMax];
    __shared__ uint32_t s_hmask[kBbHeavyMax];
    __shared__ uint32_t s_nearany;
    __shared__ double s_wmax[S], s_thr[S];
    __shared__ unsigned long long s_wkey[S], s_farmin[S];
    __shared__ int64_t s_src[S];
    __shared__ unsigned long long s_relax;
    __shared__ int32_t w_pre[NW][65];
    __shared__ int64_t w_beg[NW][64];
    __shared__ uint32_t w_m[NW][64];
    __shared__ double w_d[NW][64][S];
    unsigned long long *dist = dist_all + (int64_t)blockIdx.x * n * S;
    uint32_t *qmask = qmask_all + (int64_t)blockIdx.x * n;
    int32_t *fa = fr_all + (int64_t)blockIdx.x * 2 * n;
    int32_t *fb = fa + n;
    uint32_t *fm = fm_all + (int64_t)blockIdx.x * n;
    int32_t *touched = touched_all + (int64_t)blockIdx.x * n;
    int32_t *farA = far_all + (int64_t)blockIdx.x * 2 * n, *farB = farA + n;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const double thr0 = delta > 0.0 ? delta : __longlong_as_double((long long)kInfBits);
    if (threadIdx.x == 0) s_relax = 0;
    unsigned long long relax = 0;
    const int64_t nbatch = PAIR ? nsrc : (nsrc + S - 1) / S;
    __shared__ int64_t s_pcol;
    // batches taken in order from a global counter as workgroups free up (batch_next;
    // null: static striding), so the long searches at the end of the order do not
    // leave workgroups idle behind a fixed share
    // batches [b0, b1) of the processing order (b1 <= nbatch), this part's every
    // nparts-th one: the j-th taken is b0 + part + j * nparts
    __shared__ long long s_bq;
    if (threadIdx.x == 0) s_bq = batch_next ? (long long)atomicAdd(batch_next, 1ull) : (long long)blockIdx.x;
    __syncthreads();
    for (int64_t bj = s_bq, bq = b0 + part + bj * nparts; bq < b1; bj = s_bq, bq = b0 + part + bj * nparts) {
        // rev: the batches from the last (the sources are in node order, i.e. by
        // descending column count after the relabeling)
        const int64_t bi = rev ? nbatch - 1 - bq : bq;
        // GSPARSE_BB_TRACE: the batch's start / end on the constant clock and workgroup
        const unsigned long long tb0 = trace ? (unsigned long long)wall_clock64() : 0ull;
        if (threadIdx.x < S) {
            if constexpr (PAIR) {
                const int64_t i = sources[bi];
                s_src[threadIdx.x] = threadIdx.x == 0 ? src[i] : dst[i];
                if (threadIdx.x == 0) s_pcol = i;
            } else {
                const int64_t si = bi * S + threadIdx.x;
                s_src[threadIdx.x] = si < nsrc ? sources[si] : -1;
            }
            s_wkey[threadIdx.x] = 0ull;
            s_thr[threadIdx.x] = thr0;
            s_farmin[threadIdx.x] = kInfBits;
        }
        __syncthreads();
        if constexpr (PAIR) {  // the radius: half the larger of the pair's open weights
            if (threadIdx.x == 0) {
                const int64_t i = s_pcol, u = s_src[0], v = s_src[1];
                double wm = w[i];
                const int64_t rp = rpos[i];
                if (rp >= 0) {
                    const uint64_t rkey = (uint64_t)v * (uint64_t)n + (uint64_t)u;
                    for (int64_t p = rp; p < E && skeys[p] == rkey; ++p)  // the open ones only
                        if (state[sidx[p]] == 0) wm = w[sidx[p]] > wm ? w[sidx[p]] : wm;
                }
                const double r = wm * (1.0 + 8.0 * mrg) * 0.5;
                // an end that is a (complete) landmark: its labels are exact already
                const bool skip = lmflag && (lmflag[u] || lmflag[v]);
                s_wkey[0] = s_wkey[1] = skip ? 0ull : dkey(r);
            }
            __syncthreads();
        } else
        // largest unresolved target weight of each source (none: nothing to decide)
        {
            unsigned long long lm[S];
#pragma unroll
            for (int k = 0; k < S; ++k) {
                lm[k] = 0ull;
                const int64_t u = s_src[k];
                if (u >= 0)
                    for (int64_t j = optr[u] + threadIdx.x; j < optr[u + 1]; j += NT) {
                        const int64_t idx = order[j];
                        if (state[idx] == 0) {
                            const unsigned long long kk = dkey(w[idx]);
                            lm[k] = kk > lm[k] ? kk : lm[k];
                        }
                    }
            }
            bb_block_max_s<S>(lm, s_wkey);
        }
        if (threadIdx.x < S)
            s_wmax[threadIdx.x] = s_wkey[threadIdx.x] ? dkey_val(s_wkey[threadIdx.x]) : -1.0;
        __syncthreads();
        if (trace && threadIdx.x == 0) {  // the batch's largest bound and its column count
            double bm = -1.0;
            long long nc = 0;
            for (int k = 0; k < S; ++k) {
                bm = s_wmax[k] > bm ? s_wmax[k] : bm;
                if (s_src[k] >= 0) nc += optr[s_src[k] + 1] - optr[s_src[k]];
            }
            trace[6 * bj + 3] = (unsigned long long)__double_as_longlong(bm);
            trace[6 * bj + 4] = (unsigned long long)nc;
        }
        const unsigned long long relax0 = relax;
        // seed: every live source at its own node (sources are distinct nodes)
        if (threadIdx.x == 0) {
            int f = 0;
            for (int k = 0; k < S; ++k) {
                if (s_src[k] < 0 || s_wmax[k] < 0.0) continue;
                const int32_t u = (int32_t)s_src[k];
                dist[(int64_t)u * S + k] = 0ull;
                qmask[u] = (1u << k) | kQMaskTouched;
                fa[f] = u;
                touched[f] = u;
                ++f;
            }
            s_fcount = f;
            s_ncount = 0;
            s_tcount = f;
            s_nfar = 0;
            s_farleft = 0;
            s_nearany = 0;
            s_nbig = 0;
            s_amin = kInfBits;
        }
        __syncthreads();
        int32_t *cur = fa, *nxt = fb;
        uint32_t nearacc = 0;  // sources this lane queued near in the round
        while (true) {
            const int fc = s_fcount;
            if (fc == 0 && !s_farleft) break;
            // the bounds in registers (8 sources or fewer), else read from LDS per relaxation
            constexpr int SW = S <= 8 ? S : 1;
            double wmax[SW];
#pragma unroll
            for (int k = 0; k < SW; ++k) wmax[k] = s_wmax[k];
            auto wmax_of = [&](int k) -> double {
                if constexpr (S <= 8) return wmax[k];
                else return s_wmax[k];
            };
            if (threadIdx.x == 0) s_nheavy = 0;
            __syncthreads();
            // heavy frontier nodes (more than kBbHeavy entries: the R-MAT hubs) are taken
            // out of the per-wave chunks and expanded by the whole workgroup below, so one
            // wave does not walk a hub's list while the others wait at the barrier
            for (int f = threadIdx.x; f < fc; f += NT) {
                const int32_t x = cur[f];
                uint32_t m = atomicAnd(&qmask[x], ~QS) & QS;
                if (m && gp[x + 1] - gp[x] > kBbHeavy) {
                    const int h = atomicAdd(&s_nheavy, 1);
                    if (h < kBbHeavyMax) {
                        s_heavy[h] = x;
                        s_hmask[h] = m;
                        m = 0;
                    }
                }
                fm[f] = m;
            }
            __syncthreads();
            for (int f0 = wv * 64; f0 < fc; f0 += NT) {
                const int f = f0 + lane;
                int deg = 0;
                int64_t b = 0;
                uint32_t m = 0;
                if (f < fc) {
                    const int32_t x = cur[f];
                    m = fm[f];
                    b = gp[x];
                    deg = m ? (int)(gp[x + 1] - b) : 0;
#pragma unroll
                    for (int k = 0; k < S; ++k)
                        w_d[wv][lane][k] = __longlong_as_double((long long)__hip_atomic_load(
                            &dist[(int64_t)x * S + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                }
                int incl = deg;
                for (int off = 1; off < 64; off <<= 1) {
                    const int t = __shfl_up(incl, off, 64);
                    if (lane >= off) incl += t;
                }
                const int total = __shfl(incl, 63, 64);
                w_pre[wv][lane + 1] = incl;
                if (lane == 0) w_pre[wv][0] = 0;
                w_beg[wv][lane] = b;
                w_m[wv][lane] = m;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                constexpr int U = S >= 16 ? 1 : S >= 8 ? 2 : 4;  // edges per lane per trip, all loads in flight
                for (int e0 = 0; e0 < total; e0 += 64 * U) {
                    int lo[U];
                    uint32_t mm[U];
                    double we[U];
                    int32_t y[U];
                    unsigned long long cd[U][S];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int e = e0 + u * 64 + lane;
                        const int ec = e < total ? e : 0;
                        int a = 0, z = 63;  // largest k with w_pre[k] <= ec
                        while (a < z) {
                            const int mid = (a + z + 1) >> 1;
                            if (w_pre[wv][mid] <= ec) a = mid;
                            else z = mid - 1;
                        }
                        lo[u] = a;
                        const int64_t ei = w_beg[wv][a] + (ec - w_pre[wv][a]);
                        mm[u] = e < total ? w_m[wv][a] : 0u;
                        we[u] = gw[ei];
                        y[u] = gi[ei];
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u)
#pragma unroll
                        for (int k = 0; k < S; ++k)
                            cd[u][k] = ((mm[u] >> k) & 1u)
                                           ? __hip_atomic_load(&dist[(int64_t)y[u] * S + k],
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)
                                           : 0ull;
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                    uint32_t imp = 0, fimp = 0;
                    bool btouch = false;  // PAIR: a label set beyond the radius
                    // PAIR: complete landmarks are reached, never expanded (their labels
                    // bound the paths through them, min_l D_l(u) + D_l(v))
                    const bool blk = PAIR && lmflag && mm[u] && lmflag[y[u]];
#pragma unroll
                    for (int k = 0; k < S; ++k) {
                        if (!((mm[u] >> k) & 1u)) continue;
                        ++relax;
                        const double nd = w_d[wv][lo[u]][k] + we[u];
                        if (!(nd <= wmax_of(k)) || blk) {
                            // PAIR: kept (a T label of the certificate), never expanded
                            if constexpr (PAIR) {
                                const unsigned long long nb = (unsigned long long)__double_as_longlong(nd);
                                if (nb < cd[u][k]) {
                                    atomicMin(&dist[(int64_t)y[u] * S + k], nb);
                                    btouch = true;
                                }
                            }
                            continue;
                        }
                        const unsigned long long nb = (unsigned long long)__double_as_longlong(nd);
                        if (nb >= cd[u][k]) continue;
                        if (bb_min_improves(&dist[(int64_t)y[u] * S + k], nb)) {
                            if (!NF || nd < s_thr[k]) {  // LDS: read on improvements only
                                imp |= 1u << k;
                            } else {
                                fimp |= 1u << (kQMaskFarShift + k);
                                atomicMin(&s_farmin[k], nb);
                            }
                        }
                    }
                    if (imp | fimp) {  // queue y once per round; far: list it once, reset list
                        const uint32_t add = fimp ? (imp | fimp | kQMaskFarListed | kQMaskTouched) : imp;
                        const uint32_t om = atomicOr(&qmask[y[u]], add);
                        if (imp && (om & QS) == 0) {
                            const int q = atomicAdd(&s_ncount, 1);
                            nxt[q] = y[u];
                        }
                        if (fimp && !(om & kQMaskFarListed)) farA[atomicAdd(&s_nfar, 1)] = y[u];
                        if (fimp && !(om & kQMaskTouched)) touched[atomicAdd(&s_tcount, 1)] = y[u];
                        nearacc |= imp;
                    }
                    if (PAIR && btouch && !(atomicOr(&qmask[y[u]], kQMaskTouched) & kQMaskTouched))
                        touched[atomicAdd(&s_tcount, 1)] = y[u];
                    }
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            {
                const int nh = s_nheavy < kBbHeavyMax ? s_nheavy : kBbHeavyMax;
                for (int h = 0; h < nh; ++h) {
                    const int32_t x = s_heavy[h];
                    const uint32_t m = s_hmask[h];
                    // the hub's labels: wave 0 stages them in its w_d row 0 (free after the
                    // light chunks), every wave reads them from there
                    if (wv == 0 && lane < S)
                        w_d[0][0][lane] = ((m >> lane) & 1u) ? __longlong_as_double((long long)__hip_atomic_load(
                                                                   &dist[(int64_t)x * S + lane], __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_WORKGROUP))
                                                             : 0.0;
                    __syncthreads();
                    const int64_t e1 = gp[x + 1];
                    for (int64_t e = gp[x] + threadIdx.x; e < e1; e += NT) {
                        const int32_t y = gi[e];
                        const double we = gw[e];
                        unsigned long long cd[S];
#pragma unroll
                        for (int k = 0; k < S; ++k)
                            cd[k] = ((m >> k) & 1u) ? __hip_atomic_load(&dist[(int64_t)y * S + k], __ATOMIC_RELAXED,
                                                                        __HIP_MEMORY_SCOPE_WORKGROUP)
                                                    : 0ull;
                        uint32_t imp = 0, fimp = 0;
                        bool btouch = false;
                        const bool blk = PAIR && lmflag && lmflag[y];
#pragma unroll
                        for (int k = 0; k < S; ++k) {
                            if (!((m >> k) & 1u)) continue;
                            ++relax;
                            const double nd = w_d[0][0][k] + we;
                            if (!(nd <= wmax_of(k)) || blk) {
                                if constexpr (PAIR) {
                                    const unsigned long long nb = (unsigned long long)__double_as_longlong(nd);
                                    if (nb < cd[k]) {
                                        atomicMin(&dist[(int64_t)y * S + k], nb);
                                        btouch = true;
                                    }
                                }
                                continue;
                            }
                            const unsigned long long nb = (unsigned long long)__double_as_longlong(nd);
                            if (nb >= cd[k]) continue;
                            if (bb_min_improves(&dist[(int64_t)y * S + k], nb)) {
                                if (!NF || nd < s_thr[k]) {
                                    imp |= 1u << k;
                                } else {
                                    fimp |= 1u << (kQMaskFarShift + k);
                                    atomicMin(&s_farmin[k], nb);
                                }
                            }
                        }
                        if (imp | fimp) {
                            const uint32_t add = fimp ? (imp | fimp | kQMaskFarListed | kQMaskTouched) : imp;
                            const uint32_t om = atomicOr(&qmask[y], add);
                            if (imp && (om & QS) == 0) nxt[atomicAdd(&s_ncount, 1)] = y;
                            if (fimp && !(om & kQMaskFarListed)) farA[atomicAdd(&s_nfar, 1)] = y;
                            if (fimp && !(om & kQMaskTouched)) touched[atomicAdd(&s_tcount, 1)] = y;
                            nearacc |= imp;
                        }
                        if (PAIR && btouch && !(atomicOr(&qmask[y], kQMaskTouched) & kQMaskTouched))
                            touched[atomicAdd(&s_tcount, 1)] = y;
                    }
                    __syncthreads();
                }
            }
            if (NF && delta > 0.0) {  // which sources queued anything near this round
                uint32_t v = nearacc;
                for (int off = 32; off > 0; off >>= 1) v |= __shfl_xor(v, off, 64);
                if (lane == 0 && v) atomicOr(&s_nearany, v);
                nearacc = 0;
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
            // every node improved this round is in the new frontier: the first time one
            // appears there it joins the reset list
            {
                const int nf = s_fcount;
                for (int f = threadIdx.x; f < nf; f += NT) {
                    const int32_t y = cur[f];
                    const uint32_t om = atomicOr(&qmask[y], kQMaskTouched);
                    if (!(om & kQMaskTouched)) touched[atomicAdd(&s_tcount, 1)] = y;
                }
            }
            // hook: prune targets per source, lower its bound, end when all are done
            if (threadIdx.x < S) s_wkey[threadIdx.x] = 0ull;
            __syncthreads();
            if constexpr (PAIR) {
                if (threadIdx.x < S) s_wkey[threadIdx.x] = dkey(s_wmax[threadIdx.x]);  // the radius stays
                __syncthreads();
            } else {
                unsigned long long mx[S];
#pragma unroll
                for (int k = 0; k < S; ++k) {
                    mx[k] = 0ull;
                    const int64_t u = s_src[k];
                    if (u >= 0 && s_wmax[k] >= 0.0)
                        for (int64_t j = optr[u] + threadIdx.x; j < optr[u + 1]; j += NT) {
                            const int64_t idx = order[j];
                            if (state[idx] != 0) continue;
                            const unsigned long long db = __hip_atomic_load(
                                &dist[dst[idx] * S + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                            if (db != kInfBits &&
                                w[idx] > __longlong_as_double((long long)db) + eps) {
                                bb_set(state, why, idx, 2, kWhySearchPrune);
                                continue;
                            }
                            const unsigned long long kk = dkey(w[idx]);
                            mx[k] = kk > mx[k] ? kk : mx[k];
                        }
                }
                bb_block_max_s<S>(mx, s_wkey);
            }
            __shared__ uint32_t s_refill;
            __shared__ double s_throld[S];
            if (threadIdx.x == 0) {
                bool any = false;
                for (int k = 0; k < S; ++k) {
                    s_wmax[k] = s_wkey[k] ? dkey_val(s_wkey[k]) : -1.0;
                    any = any || s_wkey[k] != 0ull;
                }
                if (!any) s_fcount = 0;
                // near-far: a source with nothing near queued and far labels pending
                // moves its threshold past the least of them
                uint32_t R = 0;
                if (NF && any && delta > 0.0)
                    for (int k = 0; k < S; ++k)
                        if (!((s_nearany >> k) & 1u) && s_farmin[k] != kInfBits) {
                            R |= 1u << k;
                            s_throld[k] = s_thr[k];
                            const double m = __longlong_as_double((long long)s_farmin[k]);
                            s_thr[k] = (m > s_thr[k] ? m : s_thr[k]) + delta;
                            s_farmin[k] = kInfBits;
                        }
                s_refill = R;
                s_nearany = 0;
                s_nfar2 = 0;
                s_farleft = any && s_nfar > 0 && (R || s_fcount > 0);
            }
            __syncthreads();
            const uint32_t R = NF ? s_refill : 0u;
            if (NF && R) {
                // far labels of the refilled sources: below the old threshold (expanded when
                // they improved) or beyond the bound -> dropped; below the new one -> the
                // frontier; the rest stay, and give the source's next least far label
                const int nf = s_nfar;
                for (int i = threadIdx.x; i < nf; i += NT) {
                    const int32_t y = farA[i];
                    const uint32_t om = __hip_atomic_load(&qmask[y], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_WORKGROUP);
                    uint32_t clear = 0, set = 0;
#pragma unroll
                    for (int k = 0; k < S; ++k) {
                        if (!((R >> k) & 1u) || !((om >> (kQMaskFarShift + k)) & 1u)) continue;
                        const unsigned long long db = __hip_atomic_load(
                            &dist[(int64_t)y * S + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        const double d = __longlong_as_double((long long)db);
                        if (!(d <= s_wmax[k]) || d < s_throld[k]) {
                            clear |= 1u << (kQMaskFarShift + k);
                        } else if (d < s_thr[k]) {
                            clear |= 1u << (kQMaskFarShift + k);
                            set |= 1u << k;
                        } else {
                            atomicMin(&s_farmin[k], db);
                        }
                    }
                    uint32_t nm = (om & ~clear) | set;
                    if (!(nm & (QS << kQMaskFarShift))) nm &= ~kQMaskFarListed;
                    __hip_atomic_store(&qmask[y], nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (set && !(om & QS)) cur[atomicAdd(&s_fcount, 1)] = y;
                    if (nm & kQMaskFarListed) farB[atomicAdd(&s_nfar2, 1)] = y;
                }
                __syncthreads();
                if (threadIdx.x == 0) {
                    s_nfar = s_nfar2;
                    s_farleft = s_nfar2 > 0;
                }
                int32_t *t = farA;
                farA = farB;
                farB = t;
                __syncthreads();
            }
        }
        if constexpr (PAIR) {
            // The balls of radius r around u and v (labels <= r exact, expanded; a label
            // beyond r is kept but never expanded: T_v(x) = min over v's ball nodes y of
            // d_v(y) + w_yx, the fold of a real v-x walk).  Every u-v path P but the edge
            // itself, of length L <= 2r (1 - 3m): x = its last node with
            // d_P(u, x) <= r (1 - 2m) and y the next lie in u's and v's balls (the labels
            // fold within m of the exact lengths; d_P(y, v) < r (1 - 4m)), so
            // d_u(x) + T_v(x) <= L (1 + 2m) (x = v: T_v(v) = 0).  x = u (P's first edge
            // leaves u's ball) is taken over u's other edges: w_uy + d_v(y), y in v's ball.
            // So M = min(min over x in u's ball but u of d_u(x) + T_v(x),
            //            min over (u, y), y != v, d_v(y) <= r of w_uy + d_v(y))
            // is at most (1 + 4m) times every such path's fold; every term is the length of
            // a real u-v walk (one through the edge itself is at least w_G: the prune below
            // then follows from d <= w_G; x = u, whose T_v may hold w_G, is excluded).  A
            // column (u, v) or (v, u) of weight w <= 2r (1 - 5m) (a longer path folds to
            // more than 2r (1 - 4m) > w):
            //  * w > fl(w_G + eps) (its own edge in G is shorter): prune (d <= w_G);
            //  * M (1 - 5m) >= w: every alternative path folds to >= w, and w <=
            //    fl(w_G + eps): keep (the reference's w <= fl(d + eps));
            //  * (M (1 + 4m) + eps)(1 + m) < w: a shorter path exists: prune.
            // Otherwise the column stays open for the searches.
            const int64_t u = s_src[0], v = s_src[1];
            const double r = s_wmax[0];
            double mloc = __longlong_as_double((long long)kInfBits);
            // paths through a blocked landmark l: at least D_l(u) + D_l(v) (its exact labels)
            if (lmflag)
                for (int l = threadIdx.x; l < K; l += NT)
                    if (lcomp[l]) {
                        const double t2 = (LD[u * K + l] + LD[v * K + l]) * (1.0 - 2.0 * mrg);
                        mloc = t2 < mloc ? t2 : mloc;
                    }
            const int tc = s_tcount;
            for (int t = threadIdx.x; t < tc; t += NT) {
                const int32_t x = touched[t];
                if (x == (int32_t)u) continue;  // u's first edges: below
                const double du = __longlong_as_double((long long)__hip_atomic_load(
                    &dist[(int64_t)x * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                const unsigned long long bv = __hip_atomic_load(&dist[(int64_t)x * 2 + 1], __ATOMIC_RELAXED,
                                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                if (du <= r && bv != kInfBits) {
                    const double t2 = du + __longlong_as_double((long long)bv);
                    mloc = t2 < mloc ? t2 : mloc;
                }
            }
            for (int64_t e = gp[u] + threadIdx.x; e < gp[u + 1]; e += NT) {
                const int32_t y = gi[e];
                if (y == (int32_t)v) continue;
                const double dv = __longlong_as_double((long long)__hip_atomic_load(
                    &dist[(int64_t)y * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                if (dv <= r) {
                    const double t2 = gw[e] + dv;
                    mloc = t2 < mloc ? t2 : mloc;
                }
            }
            for (int off = 32; off > 0; off >>= 1) {
                const double o = __shfl_xor(mloc, off, 64);
                mloc = o < mloc ? o : mloc;
            }
            if ((threadIdx.x & 63) == 0)  // mloc >= 0: its bits order as the values
                atomicMin(&s_amin, (unsigned long long)__double_as_longlong(mloc));
            __syncthreads();
            if (threadIdx.x == 0 && r >= 0.0) {
                const double M = __longlong_as_double((long long)s_amin);
                // w_G(u, v): v in the shorter of the two sorted lists
                const int64_t du = gp[u + 1] - gp[u], dvv = gp[v + 1] - gp[v];
                const bool us = du <= dvv;
                int64_t lo = us ? gp[u] : gp[v], hi = us ? gp[u + 1] : gp[v + 1];
                const int64_t end = hi;
                const int32_t key = (int32_t)(us ? v : u);
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (gi[mid] < key) lo = mid + 1;
                    else hi = mid;
                }
                const bool has = lo < end && gi[lo] == key;
                const double wg = has ? gw[lo] : 0.0;
                auto decide = [&](int64_t c) {
                    if (state[c] != 0) return;
                    const double wc = w[c];
                    if (!(wc <= 2.0 * r * (1.0 - 5.0 * mrg))) return;
                    if (has && wc > wg + eps) bb_set(state, why, c, 2, kWhyMitm);
                    else if (M * (1.0 - 5.0 * mrg) >= wc) bb_set(state, why, c, 1, kWhyMitm);
                    else if ((M * (1.0 + 4.0 * mrg) + eps) * (1.0 + mrg) < wc) bb_set(state, why, c, 2, kWhyMitm);
                };
                decide(s_pcol);
                const int64_t rp = rpos[s_pcol];
                if (rp >= 0) {
                    const uint64_t rkey = (uint64_t)v * (uint64_t)n + (uint64_t)u;
                    for (int64_t p = rp; p < E && skeys[p] == rkey; ++p) decide(sidx[p]);
                }
            }
            if (threadIdx.x == 0) s_amin = kInfBits;
            __syncthreads();
        } else {
        // classify each source's unresolved targets; with cross != 0 also the reverse
        // columns (v, u) still open, from u's label of v (bb_cross_decide)
        for (int k = 0; k < S; ++k) {
            const int64_t u = s_src[k];
            if (u < 0) continue;
            const double bk = s_wmax[k];  // >= 0: u's search ran dry within this bound
            for (int64_t j = optr[u] + threadIdx.x; j < optr[u + 1]; j += NT) {
                const int64_t idx = order[j];
                const uint8_t st0 = state[idx];
                if (st0 != 0 && !cross) continue;
                const int64_t v = dst[idx];
                const unsigned long long db = __hip_atomic_load(
                    &dist[v * S + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const double d = __longlong_as_double((long long)db);
                if (st0 == 0) {
                    const bool keep = (db == kInfBits) || (w[idx] <= d + eps);
                    bb_set(state, why, idx, keep ? 1 : 2, keep ? kWhySearchKeep : kWhySearchPrune);
                }
                if (cross &&
                    bb_cross_decide<S>(skeys, sidx, rpos[idx], u, v, n, E, k, db, bk, mrg, eps, w, gp, gi,
                                       gw, dist, state, why)) {
                    const int q = atomicAdd(&s_nbig, 1);
                    if (q < kBbCrossBig) s_big[q] = (idx << 4) | k;
                }
            }
        }
        __syncthreads();
        // deferred exact reverse decisions (targets of many neighbours): the workgroup
        // takes the lower bound A over v's neighbours together (bb_cross_decide's rule)
        {
            const int nbg = s_nbig < kBbCrossBig ? s_nbig : kBbCrossBig;
            for (int q = 0; q < nbg; ++q) {
                const int64_t idx = s_big[q] >> 4;
                const int k = (int)(s_big[q] & 15);
                const int64_t u = s_src[k], v = dst[idx];
                const double bk = s_wmax[k];
                double a = __longlong_as_double((long long)kInfBits);
                for (int64_t e = gp[v] + threadIdx.x; e < gp[v + 1]; e += NT) {
                    const int32_t x = gi[e];
                    if (x == u) continue;
                    const unsigned long long bx = __hip_atomic_load(&dist[(int64_t)x * S + k], __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_WORKGROUP);
                    const double dx = __longlong_as_double((long long)bx);
                    const double lb = ((bx != kInfBits && dx <= bk) ? dx : bk) + gw[e];
                    a = lb < a ? lb : a;
                }
                for (int off = 32; off > 0; off >>= 1) {
                    const double o = __shfl_xor(a, off, 64);
                    a = o < a ? o : a;
                }
                if ((threadIdx.x & 63) == 0)  // a >= 0: its bits order as the values
                    atomicMin(&s_amin, (unsigned long long)__double_as_longlong(a));
                __syncthreads();
                if (threadIdx.x == 0) {
                    const double A = __longlong_as_double((long long)s_amin);
                    const double D = __longlong_as_double((long long)__hip_atomic_load(
                        &dist[v * S + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
                    if (A * (1.0 - 3.0 * mrg) > D) {
                        const uint64_t rkey = (uint64_t)v * (uint64_t)n + (uint64_t)u;
                        for (int64_t p = rpos[idx]; p < E && skeys[p] == rkey; ++p) {
                            const int64_t r = sidx[p];
                            if (state[r] == 0) bb_set(state, why, r, w[r] <= D + eps ? 1 : 2, kWhyRevExact);
                        }
                    }
                    s_amin = kInfBits;
                }
                __syncthreads();
            }
        }
        }  // !PAIR
        __syncthreads();
        if (trace && relax != relax0) atomicAdd(&trace[6 * bj + 5], relax - relax0);
        const int tc = s_tcount;
        for (int t = threadIdx.x; t < tc; t += NT) {
            const int32_t y = touched[t];
#pragma unroll
            for (int k = 0; k < S; ++k) dist[(int64_t)y * S + k] = kInfBits;
            qmask[y] = 0u;
        }
        if (threadIdx.x == 0) {
            if (trace) {
                trace[6 * bj] = tb0;
                trace[6 * bj + 1] = (unsigned long long)wall_clock64();
                trace[6 * bj + 2] = blockIdx.x;
            }
            s_bq = batch_next ? (long long)atomicAdd(batch_next, 1ull) : (long long)(bj + gridDim.x);
        }
        __syncthreads();
    }
    atomicAdd(&s_relax, relax);
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(relax_total, s_relax);
}

// Full searches from K landmarks: D[x*K + l] = d_fl(landmark l, x) (+inf if
// unreachable).  One workgroup per landmark; the landmarks l = lpart (mod lparts)
// only (the staged multi-rank form splits them over the ranks; D is +inf and
// complete 0 for the others, which the exchange's min / max fills in).
__global__ void __launch_bounds__(1024) k_bb_landmarks(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, const int32_t *__restrict__ lm, int K, int lpart, int lparts, int max_rounds,
    double *__restrict__ D,
    int32_t *__restrict__ complete, unsigned long long *__restrict__ dist_all,
    int32_t *__restrict__ qflag_all, int32_t *__restrict__ fr_all,
    int32_t *__restrict__ touched_all) {
    __shared__ int s_fcount, s_ncount, s_tcount, s_rounds, s_cut;
    __shared__ double s_inf;
    unsigned long long *dist = dist_all + (int64_t)blockIdx.x * n;
    int32_t *qflag = qflag_all + (int64_t)blockIdx.x * n;
    int32_t *fa = fr_all + (int64_t)blockIdx.x * 2 * n;
    int32_t *fb = fa + n;
    int32_t *touched = touched_all + (int64_t)blockIdx.x * n;
    unsigned long long relax = 0;
    for (int l = lpart + (int)blockIdx.x * lparts; l < K; l += (int)gridDim.x * lparts) {
        if (threadIdx.x == 0) {
            s_fcount = 1;
            s_ncount = 0;
            s_tcount = 1;
            s_inf = __builtin_inf();
            s_rounds = 0;
            s_cut = 0;
        }
        __syncthreads();
        // capped at max_rounds frontier rounds (long-diameter graphs): the
        // distances are then upper bounds only -- complete[l] = 0
        bb_search(gp, gi, gw, lm[l], s_inf, dist, qflag, fa, fb, touched, s_fcount, s_ncount,
                  s_tcount, relax, [&] {
                      if (threadIdx.x == 0 && ++s_rounds >= max_rounds && s_fcount > 0) {
                          s_fcount = 0;
                          s_cut = 1;
                      }
                      __syncthreads();
                  });
        if (threadIdx.x == 0) complete[l] = !s_cut;
        const int tc = s_tcount;
        for (int t = threadIdx.x; t < tc; t += blockDim.x) {
            const int32_t y = touched[t];
            D[(int64_t)y * K + l] = __longlong_as_double((long long)dist[y]);
            dist[y] = kInfBits;
            qflag[y] = 0;
        }
        __syncthreads();
    }
}

// The same landmark searches spread over the whole GPU (large graphs): W workgroups per
// landmark and one launch per frontier round -- the launch boundary is the round's
// barrier and makes every label of the round visible to every CU of the next (a
// single-workgroup search is one CU's throughput: 48 of them took 21.8 ms on RMAT-18,
// and 6 per rank as long).  Labels are D's own words (IEEE bits; non-negative doubles
// order as their bits), lowered by device-scope atomicMin; a label read for a check may
// be older than this round's atomics, which costs a redundant atomic, never a missed
// improvement (every improvement queues its node for the next round).  Frontier items
// are (node, chunk of kLmChunk edges), so a hub's list is split over the waves of all W
// workgroups; a node is queued for round r + 1 once (atomicMax of its round stamp).
// The fixpoint -- the least one of d(y) = min_x fl(d(x) + w(x, y)) -- is the one the
// one-workgroup search reaches; complete[l] = 0 when a landmark still had a frontier
// after max_rounds rounds.
static constexpr int kLmChunk = 256;
// per landmark j (local index): counters cnt[4 j + (r mod 3)] = items of round r
__global__ void k_lm_init(const int64_t *__restrict__ gp, const int32_t *__restrict__ lm, int K,
                          int lpart, int lparts, int mine, int64_t cap,
                          unsigned long long *__restrict__ D, uint64_t *__restrict__ items,
                          int32_t *__restrict__ cnt) {
    const int j = blockIdx.x;
    if (j >= mine) return;
    const int l = lpart + j * lparts;
    const int32_t s = lm[l];
    const int64_t d = gp[s + 1] - gp[s];
    const int nch = (int)((d + kLmChunk - 1) / kLmChunk);
    uint64_t *cur = items + (size_t)j * 2 * cap;
    for (int c = threadIdx.x; c < nch; c += blockDim.x) cur[c] = (uint64_t)(uint32_t)s << 32 | (uint32_t)c;
    if (threadIdx.x == 0) {
        D[(int64_t)s * K + l] = 0ull;  // +0.0
        cnt[4 * j] = nch;
        cnt[4 * j + 1] = 0;
        cnt[4 * j + 2] = 0;
    }
}

template <int NT>
__global__ void __launch_bounds__(NT) k_lm_round(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, int K, int lpart, int lparts, int W, int r, int64_t cap,
    unsigned long long *__restrict__ D, uint64_t *__restrict__ items, uint32_t *__restrict__ stamp,
    int32_t *__restrict__ cnt) {
    constexpr int NW = NT / 64;
    const int j = blockIdx.x / W, wb = blockIdx.x - j * W;
    const int l = lpart + j * lparts;
    int32_t *cj = cnt + 4 * j;
    const int fc = cj[r % 3];
    // the counter of round r + 2 was last read in round r - 1
    if (wb == 0 && threadIdx.x == 0) cj[(r + 2) % 3] = 0;
    if (fc == 0) return;  // workgroup-uniform
    const uint64_t *cur = items + ((size_t)j * 2 + (r & 1)) * cap;
    uint64_t *nxt = items + ((size_t)j * 2 + ((r + 1) & 1)) * cap;
    uint32_t *st = stamp + (size_t)j * n;
    int32_t *cn = cj + (r + 1) % 3;
    const uint32_t rn = (uint32_t)r + 1u;
    __shared__ int32_t w_pre[NW][65];
    __shared__ int64_t w_beg[NW][64];
    __shared__ double w_d[NW][64];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    // items per wave: up to 64, fewer when the frontier is short (a hub's chunks in the
    // first rounds would otherwise all fall to a few waves)
    const int per = max(1, min(64, (fc + W * NW - 1) / (W * NW)));
    for (int f0 = (wb * NW + wv) * per; f0 < fc; f0 += W * NW * per) {
        const int f = f0 + lane;
        int deg = 0;
        int64_t b = 0;
        double dx = 0.0;
        if (lane < per && f < fc) {
            const uint64_t it = cur[f];
            const int32_t x = (int32_t)(it >> 32);
            const int64_t a = gp[x] + (int64_t)(uint32_t)it * kLmChunk, e1 = gp[x + 1];
            b = a;
            deg = (int)(e1 - a < kLmChunk ? e1 - a : kLmChunk);
            dx = __longlong_as_double((long long)D[(int64_t)x * K + l]);
        }
        int incl = deg;
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off, 64);
            if (lane >= off) incl += t;
        }
        const int total = __shfl(incl, 63, 64);
        w_pre[wv][lane + 1] = incl;
        if (lane == 0) w_pre[wv][0] = 0;
        w_beg[wv][lane] = b;
        w_d[wv][lane] = dx;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        constexpr int U = 4;  // edges per lane per trip, all loads in flight
        for (int e0 = 0; e0 < total; e0 += 64 * U) {
            int32_t y[U];
            unsigned long long nb[U], cd[U];
            bool go[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = e0 + u * 64 + lane;
                go[u] = e < total;
                const int ec = go[u] ? e : 0;
                int lo = 0, hi = 63;  // largest k with w_pre[k] <= ec
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (w_pre[wv][mid] <= ec) lo = mid;
                    else hi = mid - 1;
                }
                const int64_t ei = w_beg[wv][lo] + (ec - w_pre[wv][lo]);
                nb[u] = (unsigned long long)__double_as_longlong(w_d[wv][lo] + gw[ei]);
                y[u] = gi[ei];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) cd[u] = go[u] ? D[(int64_t)y[u] * K + l] : 0ull;
            // the U atomics of a lane in flight together, then the stamps of the improved
#pragma unroll
            for (int u = 0; u < U; ++u) {
                go[u] = go[u] && nb[u] < cd[u];
                cd[u] = go[u] ? atomicMin(&D[(int64_t)y[u] * K + l], nb[u]) : 0ull;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) go[u] = go[u] && nb[u] < cd[u] && atomicMax(&st[y[u]], rn) < rn;
            int nch[U], mine = 0;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                nch[u] = go[u] ? (int)((gp[y[u] + 1] - gp[y[u]] + kLmChunk - 1) / kLmChunk) : 0;
                mine += nch[u];
            }
            // one counter add per wave and trip (a single word takes ~90 adds per us)
            int incl = mine;
            for (int off = 1; off < 64; off <<= 1) {
                const int t = __shfl_up(incl, off, 64);
                if (lane >= off) incl += t;
            }
            const int wtot = __shfl(incl, 63, 64);
            if (wtot) {
                int base = 0;
                if (lane == 63) base = atomicAdd(cn, wtot);
                int q = __shfl(base, 63, 64) + incl - mine;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    for (int c = 0; c < nch[u]; ++c) nxt[q++] = (uint64_t)(uint32_t)y[u] << 32 | (uint32_t)c;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// sum of the next round's item counts of every landmark into *tot; complete flags
// (final: the counts of round r)
__global__ void k_lm_count(const int32_t *__restrict__ cnt, int mine, int r, int lpart, int lparts,
                           unsigned long long *__restrict__ tot, int32_t *__restrict__ complete,
                           int final) {
    unsigned long long s = 0;
    for (int j = threadIdx.x; j < mine; j += blockDim.x) {
        const int c = cnt[4 * j + r % 3];
        s += (unsigned long long)c;
        if (final) complete[lpart + j * lparts] = c == 0;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(tot, s);
}

// Full searches for sampled node pairs (verify_geodesic_preservation,
// compute_geodesic_preservation): one workgroup per distinct source, then the
// exact distance of each of its targets (+inf when unreachable).
__global__ void __launch_bounds__(256) k_bb_pairs(
    const int64_t *__restrict__ gp, const int32_t *__restrict__ gi, const double *__restrict__ gw,
    int64_t n, const int64_t *__restrict__ srcs, const int64_t *__restrict__ qptr,
    const int64_t *__restrict__ qt, int64_t nsrc, double *__restrict__ out,
    unsigned long long *__restrict__ dist_all, int32_t *__restrict__ qflag_all,
    int32_t *__restrict__ fr_all, int32_t *__restrict__ touched_all) {
    __shared__ int s_fcount, s_ncount, s_tcount;
    __shared__ double s_inf;
    unsigned long long *dist = dist_all + (int64_t)blockIdx.x * n;
    int32_t *qflag = qflag_all + (int64_t)blockIdx.x * n;
    int32_t *fa = fr_all + (int64_t)blockIdx.x * 2 * n;
    int32_t *fb = fa + n;
    int32_t *touched = touched_all + (int64_t)blockIdx.x * n;
    unsigned long long relax = 0;
    for (int64_t si = blockIdx.x; si < nsrc; si += gridDim.x) {
        if (threadIdx.x == 0) {
            s_fcount = 1;
            s_ncount = 0;
            s_tcount = 1;
            s_inf = __builtin_inf();
        }
        __syncthreads();
        bb_search(gp, gi, gw, (int32_t)srcs[si], s_inf, dist, qflag, fa, fb, touched, s_fcount,
                  s_ncount, s_tcount, relax, [&] { __syncthreads(); });
        for (int64_t q = qptr[si] + threadIdx.x; q < qptr[si + 1]; q += blockDim.x)
            out[q] = __longlong_as_double((long long)dist[qt[q]]);
        __syncthreads();
        const int tc = s_tcount;
        for (int t = threadIdx.x; t < tc; t += blockDim.x) {
            const int32_t y = touched[t];
            dist[y] = kInfBits;
            qflag[y] = 0;
        }
        __syncthreads();
    }
}

// Certificates for unresolved columns (state 0), each implying the exact
// comparison w <= fl(d + eps) the reference makes (d = the fl left-fold
// Dijkstra distance; fl sums of <= 2^31 terms are within 1e-9 relative of the
// exact path sums, which the margins below absorb):
//  * an endpoint of degree 1 in G whose only neighbour is the other one: every
//    path starts or ends with that edge, so d = w_G(u,v) exactly;
//  * landmark upper bound: the walk u -> l -> v has fold <= (D_l(u)+D_l(v))(1+m),
//    so w > fl(that + eps) proves w > fl(d + eps): prune;
//  * landmark lower bound: d >= |D_l(u)-D_l(v)| - m (D_l(u)+D_l(v)), so
//    w <= that proves w <= d <= fl(d + eps): keep; D_l(u) finite with D_l(v)
//    infinite (or the reverse) means u and v are disconnected: d = inf, keep.
//  * local bounds (mw != null): every u-v path but the edge itself starts with
//    another edge of u and ends with another edge of v, so its fold is at least
//    LB = fl(mu' + mv') (1 - 2m), mu' / mv' the least weights of u's / v's other
//    G edges (+inf: none).  With the edge in G (weight w_G, d <= w_G):
//    w > fl(w_G + eps) proves w > fl(d + eps): prune; else w <= LB proves
//    w <= fl(d + eps) whichever path is shortest: keep.  Without it every path is
//    another one: w <= LB keeps.  (A column whose endpoint's edges all cost far more
//    than the column -- the Jaccard-0 edges of R-MAT -- is kept here instead of by a
//    search exhausting the giant component.)
// m = max(1e-8, 8 n 2^-53) bounds the relative rounding of folds over simple
// paths (< n terms each, two of them per walk).
// per node of G: its least edge weight mw[2x] and the second least mw[2x + 1] (equal
// when tied, +inf when missing), ma[x] the neighbour of the least; one wave per node
__global__ void k_bb_minw(const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                          const double *__restrict__ gw, int64_t n, double *__restrict__ mw,
                          int32_t *__restrict__ ma) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const double inf = __builtin_inf();
    for (int64_t x = w0; x < n; x += nw) {
        double m1 = inf, m2 = inf;
        int32_t a1 = 0x7fffffff;
        for (int64_t e = gp[x] + lane; e < gp[x + 1]; e += 64) {
            const double we = gw[e];
            const int32_t y = gi[e];
            if (we < m1 || (we == m1 && y < a1)) {
                m2 = m1;
                m1 = we;
                a1 = y;
            } else if (we < m2) {
                m2 = we;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {  // merge the lanes' (least, neighbour, second)
            const double o1 = __shfl_xor(m1, off, 64), o2 = __shfl_xor(m2, off, 64);
            const int32_t oa = __shfl_xor(a1, off, 64);
            if (o1 < m1 || (o1 == m1 && oa < a1)) {
                m2 = m1 < o2 ? m1 : o2;
                m1 = o1;
                a1 = oa;
            } else {
                m2 = o1 < m2 ? o1 : m2;
            }
        }
        if (lane == 0) {
            mw[2 * x] = m1;
            mw[2 * x + 1] = m2;
            ma[x] = a1;
        }
    }
}

// per node u: the least of w_ua + (a's least edge weight but (a, u)) over u's neighbours
// a, aw[2u], its a in aa[u], the second least aw[2u + 1] (k_bb_witness's 3-edge bound);
// one wave per node
__global__ void k_bb_minw2(const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                           const double *__restrict__ gw, int64_t n, const double *__restrict__ mw,
                           const int32_t *__restrict__ ma, double *__restrict__ aw,
                           int32_t *__restrict__ aa) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    const double inf = __builtin_inf();
    for (int64_t x = w0; x < n; x += nw) {
        double m1 = inf, m2 = inf;
        int32_t a1 = 0x7fffffff;
        for (int64_t e = gp[x] + lane; e < gp[x + 1]; e += 64) {
            const int32_t y = gi[e];
            const double ve = gw[e] + (ma[y] == (int32_t)x ? mw[2 * y + 1] : mw[2 * y]);
            if (ve < m1 || (ve == m1 && y < a1)) {
                m2 = m1;
                m1 = ve;
                a1 = y;
            } else if (ve < m2) {
                m2 = ve;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const double o1 = __shfl_xor(m1, off, 64), o2 = __shfl_xor(m2, off, 64);
            const int32_t oa = __shfl_xor(a1, off, 64);
            if (o1 < m1 || (o1 == m1 && oa < a1)) {
                m2 = m1 < o2 ? m1 : o2;
                m1 = o1;
                a1 = oa;
            } else {
                m2 = o1 < m2 ? o1 : m2;
            }
        }
        if (lane == 0) {
            aw[2 * x] = m1;
            aw[2 * x + 1] = m2;
            aa[x] = a1;
        }
    }
}

__global__ void k_bb_certify(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                             const double *__restrict__ w, int64_t c0, int64_t c1,
                             const int64_t *__restrict__ gp, const int32_t *__restrict__ gi,
                             const double *__restrict__ gw, const double *__restrict__ D,
                             const int32_t *__restrict__ complete, int K, double eps, double m,
                             const double *__restrict__ mw, const int32_t *__restrict__ ma,
                             int part, int nparts, uint8_t *__restrict__ state,
                             uint8_t *__restrict__ why) {
    for (int64_t i = c0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c1;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (state[i] != 0) continue;  // decided, or another part's column (3)
        const int64_t u = src[i], v = dst[i];
        // another part's column (pair form) and self-loops: k_bb_witness's
        if (u == v || (nparts > 1 && bb_col_part(u, v, nparts) != part)) continue;
        const double wi = w[i];
        const int64_t du = gp[u + 1] - gp[u], dv = gp[v + 1] - gp[v];
        if ((du == 1 && gi[gp[u]] == v) || (dv == 1 && gi[gp[v]] == u)) {
            const double wg = du == 1 && gi[gp[u]] == v ? gw[gp[u]] : gw[gp[v]];
            bb_set(state, why, i, (wi <= wg + eps) ? 1 : 2, kWhyDeg1);  // d = fl(0 + w_G) = w_G
            continue;
        }
        if (mw) {
            // w_G(u, v): v in the shorter of the two (sorted, symmetric) lists
            const bool us = du <= dv;
            int64_t lo = us ? gp[u] : gp[v], hi = us ? gp[u + 1] : gp[v + 1];
            const int32_t key = (int32_t)(us ? v : u);
            const int64_t end = hi;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (gi[mid] < key) lo = mid + 1;
                else hi = mid;
            }
            const bool has = lo < end && gi[lo] == key;
            const double mu = ma[u] == (int32_t)v ? mw[2 * u + 1] : mw[2 * u];
            const double mv = ma[v] == (int32_t)u ? mw[2 * v + 1] : mw[2 * v];
            const double lb = (mu + mv) * (1.0 - 2.0 * m);  // +inf when either is missing
            if (has && wi > gw[lo] + eps) {
                bb_set(state, why, i, 2, kWhyDirect);
                continue;
            }
            if (wi <= lb) {
                bb_set(state, why, i, 1, kWhyLocal2);
                continue;
            }
        }
        uint8_t st = 0, cls = kWhyOpen;
        for (int l = 0; l < K && !st; ++l) {
            const double a = D[u * K + l], b = D[v * K + l];
            const bool fa = a != __builtin_inf(), fb = b != __builtin_inf();
            const bool exact = complete[l] != 0;  // else D holds upper bounds only
            if (fa != fb) {
                if (exact) {
                    st = 1;  // different components
                    cls = kWhyLmComp;
                }
            } else if (fa) {
                const double ub = (a + b) * (1.0 + m);
                if (wi > ub + eps) {
                    st = 2;
                    cls = kWhyLmPrune;
                } else if (exact) {
                    const double hi = a > b ? a : b, lo = a > b ? b : a;
                    const double lb = (hi - lo) - m * (hi + lo);
                    if (wi <= lb) {
                        st = 1;
                        cls = kWhyLmKeep;
                    }
                }
            }
        }
        state[i] = st;
        if (why && st) why[i] = cls;
    }
}

__global__ void k_bb_count0(const uint8_t *__restrict__ state, int64_t E,
                            unsigned long long *__restrict__ cnt) {
    unsigned long long c = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        c += state[i] == 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off, 64);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, c);
}

__global__ void k_bb_fill_u64(unsigned long long *p, int64_t n, unsigned long long v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// sources: rows with an unresolved target (other parts' columns are marked 3)
// flag[u] = 1 for every row with an open column (flag zeroed before); one thread per
// column (a thread per row walked a hub's 10^4-10^5 columns alone: 3.3 ms on RMAT-18)
__global__ void k_bb_need(const int64_t *__restrict__ src, const uint8_t *__restrict__ state,
                          int64_t E, int64_t *__restrict__ flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        if (state[i] == 0) flag[src[i]] = 1;
}

__global__ void k_bb_compact(const int64_t *__restrict__ flag, const int64_t *__restrict__ pos,
                             int64_t n, int64_t *__restrict__ sources) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x)
        if (flag[u]) sources[pos[u]] = u;
}

// keep bytes of this part's columns (bb_col_part), 0 elsewhere
__global__ void k_bb_keep(const uint8_t *__restrict__ state, const int64_t *__restrict__ src,
                          const int64_t *__restrict__ dst, int64_t E, int part, int nparts,
                          uint8_t *__restrict__ keep) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        keep[i] = state[i] == 1 && bb_col_part(src[i], dst[i], nparts) == part;
}

}  // namespace gs

using namespace gs;

// Node relabeling for the searches' locality: node ids ordered by descending
// column count (hubs first, ties by id), so the labels a search touches most
// often share cache lines.  Distances, sums and decisions do not depend on the
// labels (every fold runs along the path from the source), only where the
// searches' distance slabs are read.
__global__ void k_bb_count(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                           int64_t E, unsigned long long *__restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        atomicAdd(&cnt[src[i]], 1ull);
        atomicAdd(&cnt[dst[i]], 1ull);
    }
}

// sum over columns of |src - dst| (the ids' existing locality), per-wave partials
__global__ void k_bb_gap(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                         int64_t E, unsigned long long *__restrict__ sum) {
    unsigned long long acc = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = src[i] - dst[i];
        acc += (unsigned long long)(g < 0 ? -g : g);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

__global__ void k_bb_relabel_keys(const unsigned long long *__restrict__ cnt, int64_t n,
                                  uint64_t *__restrict__ keys, int64_t *__restrict__ ids) {
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t c = cnt[x] < 0xffffffffull ? cnt[x] : 0xffffffffull;
        keys[x] = ((0xffffffffull - c) << 32) | (uint64_t)x;
        ids[x] = x;
    }
}

// landmark order: ascending ((2^32 - 1 - degree in G) << 32 | id) = by degree, high first,
// ties by id (round 5's host partial_sort over a copy of G's row pointers)
__global__ void k_bb_degkeys(const int64_t *__restrict__ gp, int64_t n, uint64_t *__restrict__ keys,
                             int64_t *__restrict__ ids) {
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t d = (uint64_t)(gp[x + 1] - gp[x]);
        keys[x] = ((0xffffffffull - (d < 0xffffffffull ? d : 0xffffffffull)) << 32) | (uint64_t)x;
        ids[x] = x;
    }
}

__global__ void k_bb_first_ids(const int64_t *__restrict__ ids, int K, int32_t *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < K) out[i] = (int32_t)ids[i];
}

__global__ void k_bb_perm(const int64_t *__restrict__ ids, int64_t n, int64_t *__restrict__ perm) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        perm[ids[i]] = i;
}

__global__ void k_bb_map(const int64_t *__restrict__ perm, const int64_t *__restrict__ a,
                         const int64_t *__restrict__ b, int64_t E, int64_t *__restrict__ ma,
                         int64_t *__restrict__ mb) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        ma[i] = perm[a[i]];
        mb[i] = perm[b[i]];
    }
}

// G of metric_backbone.py:70-79 as a symmetric CSR: the columns with s < d in
// the caller's ids (osrc/odst), keyed by the ids G is built in (src/dst), weight
// the minimum over duplicates.  misc[0] is used as the unique-edge counter,
// misc + 4 as the bad-input flag.
static void bb_build_graph(gs_ctx *c, int64_t n, int64_t E, const int64_t *dsrc, const int64_t *ddst,
                           const int64_t *osrc, const int64_t *odst, const double *dw,
                           unsigned long long *misc, int64_t *&gp, int32_t *&gi, double *&gw,
                           double *wmed = nullptr, int64_t *gnnz = nullptr) {
    hipStream_t s = c->stream;
    int *bad = (int *)(misc + 4);
    uint64_t *keys = (uint64_t *)c->buf("bb_keys").ensure(8 * E);
    int64_t *idx = (int64_t *)c->buf("bb_idx").ensure(8 * E);
    k_bb_keys<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, ddst, osrc, odst, dw, E, n, keys, idx,
                                                     bad);
    int hbad = 0;
    GS_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    GS_CHECK(!(hbad & 1), GS_EINVAL, "edge_index entry out of range [0, %lld)", (long long)n);
    GS_CHECK(!(hbad & 2), GS_EUNSUPPORTED,
             "edge weights must be non-negative and not NaN (Dijkstra contract)");
    sort_pairs_u64_i64(c, keys, idx, E, bits_for_bb((uint64_t)n * (uint64_t)n));
    uint64_t *ukeys = (uint64_t *)c->buf("bb_ukeys").ensure(16 * E);
    double *uw = (double *)c->buf("bb_uw").ensure(8 * E);
    k_bb_unique<<<grid_for(E, 256, 8192), 256, 0, s>>>(keys, idx, dw, E, n, misc, ukeys, uw);
    unsigned long long ucnt = 0;
    GS_HIP(hipMemcpyAsync(&ucnt, misc, 8, hipMemcpyDeviceToHost, s));
    GS_HIP(hipStreamSynchronize(s));
    int64_t cnt2 = 2 * (int64_t)ucnt;
    if (gnnz) *gnnz = cnt2;
    if (wmed) {  // median of <= 1023 evenly spaced unique-edge weights
        *wmed = 0.0;
        if (ucnt) {
            const int64_t m = ucnt < 1023 ? (int64_t)ucnt : 1023, stride = (int64_t)ucnt / m;
            std::vector<double> smp(m);
            GS_HIP(hipMemcpy2DAsync(smp.data(), 8, uw, 8 * stride, 8, m, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            std::nth_element(smp.begin(), smp.begin() + m / 2, smp.end());
            *wmed = smp[m / 2];
        }
    }
    // G as symmetric CSR sorted by (row, col): unique keys -> no ties in order
    int64_t *pay = (int64_t *)c->buf("bb_pay").ensure(8 * (cnt2 + 1));
    k_bb_sym_payload<<<grid_for(cnt2 + 1, 256, 8192), 256, 0, s>>>(cnt2, pay);
    sort_pairs_u64_i64(c, ukeys, pay, cnt2, bits_for_bb((uint64_t)n * (uint64_t)n));
    gp = (int64_t *)c->buf("bb_gp").ensure(8 * (n + 1));
    gi = (int32_t *)c->buf("bb_gi").ensure(4 * (cnt2 + 1));
    gw = (double *)c->buf("bb_gw").ensure(8 * (cnt2 + 1));
    if (cnt2) k_bb_gfill<<<grid_for(cnt2, 256, 8192), 256, 0, s>>>(ukeys, pay, uw, cnt2, n, gi, gw);
    k_bb_rowptr<<<grid_for(n + 1, 256, 8192), 256, 0, s>>>(ukeys, cnt2, (uint64_t)n, n, gp);
}

// ---------------------------------------------------------------------------
// Host side, in stages (the prune over N ranks).  One call of
// gs_metric_backbone runs them back to back; the multi-rank form
// (gsparse.distributed.sharded_backbone) runs them on every rank with one exchange
// between stages:
//   begin     relabel, G, columns by row, this rank's landmark searches (l = part mod N)
//             -> exchange D (min) and the completeness flags (max)
//   certify   2-hop witness + degree-1 / landmark certificates of this rank's column
//             range -> exchange the column states (max: 0 open < 1 keep < 2 prune; two
//             ranks that decide a column decide it the same way, every rule is exact)
//   plan      the sources with open columns (the same list on every rank)
//   search    batches [b0, b1) of the ascending-count order, this rank's every N-th
//             -> exchange the states; the next range starts from every rank's decisions
//             (the short searches' reverse-column decisions close most hub columns
//             before the hubs search)
//   finish    keep bytes of every column
// The legacy one-exchange form (gs_metric_backbone_part: pairs max(u, v) % N, keep
// bytes summed) runs the same stages with the pair flags.
namespace gs {
struct BbRun {
    bool begun = false, certified = false, planned = false;
    int64_t n = 0, E = 0;
    double eps = 0.0;
    int pair_part = 0, pair_nparts = 1;
    int nranks = 1;  // ranks of the staged form (the search geometry depends on it)
    const int64_t *dsrc = nullptr, *ddst = nullptr, *osrc = nullptr, *odst = nullptr;
    const double *dw = nullptr;
    int64_t *gp = nullptr;
    int32_t *gi = nullptr;
    double *gw = nullptr;
    double wmed = 0.0;
    int64_t *optr = nullptr, *order = nullptr;
    uint8_t *state = nullptr;
    // decision classes (gs_bb_classes): why[E] written beside state when why_on
    bool why_on = false;
    uint8_t *why = nullptr;
    int64_t why_E = 0;
    int K = 0;
    double *D = nullptr;
    int32_t *lcomp = nullptr;
    int64_t nsrc = 0, nbatch = 0, slabs = 0;
    int S = 1, bt = 256;
    int64_t *sources = nullptr;
    unsigned long long *dist = nullptr;
    int32_t *qflag = nullptr, *fr = nullptr, *touched = nullptr, *farl = nullptr;
    uint32_t *fm = nullptr;
    uint64_t *skeys = nullptr;
    int64_t *sidx = nullptr, *rpos = nullptr;
    int cross = 1, rev = 1;
    bool keys_ready = false;  // skeys / sidx / rpos built for this run
    bool dynamic = true;
    double delta = 0.0;
    // the search slabs hold +inf labels / zero masks between searches (every batch resets
    // what it touched): filled only when (re)allocated or grown
    void *dist_ok = nullptr, *q_ok = nullptr;
    size_t dist_ok_bytes = 0, q_ok_bytes = 0;
    unsigned long long *misc = nullptr;  // [0] unique edges, [1] relaxations, [2] batch
                                         // counter, [3] debug count; misc + 4: bad flag
    hipEvent_t tall = nullptr;           // the "metric_backbone" profile region
};
}  // namespace gs

static BbRun &bb_run(gs_ctx *c) {
    if (!c->bb) c->bb = std::make_shared<BbRun>();
    return *c->bb;
}

static void bb_begin(gs_ctx *c, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                     const double *w, int64_t nw, int loc, double eps, int lpart, int lparts,
                     int pair_part, int pair_nparts) {
    GS_CHECK(c, GS_EINVAL, "null context");
    // the reference indexes edge_weights[idx] for every column (metric_backbone.py:73-74)
    GS_CHECK(nw >= E, GS_EINDEX, "index %lld is out of bounds for axis 0 with size %lld",
             (long long)nw, (long long)nw);
    GS_CHECK(E == 0 || (src && dst && w), GS_EINVAL, "null column/weight array");
    GS_CHECK(lparts >= 1 && 0 <= lpart && lpart < lparts, GS_EINVAL, "bad part %d of %d", lpart, lparts);
    GS_CHECK(pair_nparts >= 1 && 0 <= pair_part && pair_part < pair_nparts, GS_EINVAL,
             "bad part %d of %d", pair_part, pair_nparts);
    GS_CHECK(n >= 0 && E >= 0, GS_EINVAL, "negative n/E");
    GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31");
    GS_HIP(hipSetDevice(c->device));
    BbRun &R = bb_run(c);
    R.begun = R.certified = R.planned = false;
    R.keys_ready = false;
    R.n = n;
    R.E = E;
    R.eps = eps;
    R.pair_part = pair_part;
    R.pair_nparts = pair_nparts;
    R.nranks = lparts;
    R.K = 0;
    R.nsrc = R.nbatch = 0;
    hipStream_t s = c->stream;
    // own buffers (the scorer scratch slots stay untouched)
#define BB(name) DevBuf &b_##name = c->buf("bb_" #name)
    BB(src); BB(dst); BB(w); BB(okeys); BB(order); BB(optr); BB(state); BB(flag); BB(misc);
    BB(lm); BB(land); BB(lcomp); BB(dist); BB(qflag); BB(fr); BB(touched); BB(msrc); BB(mdst);
    BB(perm);
#undef BB
    const int64_t *dsrc = (const int64_t *)to_device(c, b_src, src, sizeof(int64_t) * E, loc);
    const int64_t *ddst = (const int64_t *)to_device(c, b_dst, dst, sizeof(int64_t) * E, loc);
    const int64_t *osrc = dsrc, *odst = ddst;  // the caller's ids
    bool relabel = E > 0 && n > 1;
    if (const char *e = getenv("GSPARSE_BB_RELABEL")) relabel = relabel && atoi(e) != 0;
    // only graphs whose ids carry no locality of their own (mean |u - v| above n / 64:
    // R-MAT 0.33 n; a word chain with short chords ~2) -- relabeling a chain-ordered
    // graph by degree would scatter it (Roman-like: 2.2 -> 3.2 ms)
    if (relabel && !getenv("GSPARSE_BB_RELABEL")) {
        unsigned long long *gs = (unsigned long long *)c->buf("bb_gap").ensure(8);
        GS_HIP(hipMemsetAsync(gs, 0, 8, s));
        k_bb_gap<<<grid_for(E, 256, 2048), 256, 0, s>>>(dsrc, ddst, E, gs);
        unsigned long long hg = 0;
        GS_HIP(hipMemcpyAsync(&hg, gs, 8, hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        relabel = (double)hg / (double)E > (double)n / 64.0;
    }
    if (relabel) {
        // validate before indexing the counters with the raw ids
        int *bad0 = (int *)c->buf("bb_bad0").ensure(sizeof(int));
        GS_HIP(hipMemsetAsync(bad0, 0, sizeof(int), s));
        uint64_t *k0 = (uint64_t *)c->buf("bb_keys").ensure(8 * E);
        int64_t *i0 = (int64_t *)c->buf("bb_idx").ensure(8 * E);
        k_bb_keys<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, ddst, dsrc, ddst, (const double *)to_device(
            c, b_w, w, sizeof(double) * E, loc), E, n, k0, i0, bad0);
        int hb = 0;
        GS_HIP(hipMemcpyAsync(&hb, bad0, 4, hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        GS_CHECK(!(hb & 1), GS_EINVAL, "edge_index entry out of range [0, %lld)", (long long)n);
        auto *cnt = (unsigned long long *)b_flag.ensure(8 * (n + 1));
        GS_HIP(hipMemsetAsync(cnt, 0, 8 * (n + 1), s));
        k_bb_count<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, ddst, E, cnt);
        uint64_t *nk = (uint64_t *)b_okeys.ensure(8 * (n > E ? n : E));
        int64_t *ids = (int64_t *)b_order.ensure(8 * (n > E ? n : E));
        k_bb_relabel_keys<<<grid_for(n, 256, 8192), 256, 0, s>>>(cnt, n, nk, ids);
        sort_pairs_u64_i64(c, nk, ids, n, 64);
        int64_t *perm = (int64_t *)b_perm.ensure(8 * n);
        k_bb_perm<<<grid_for(n, 256, 8192), 256, 0, s>>>(ids, n, perm);
        int64_t *ms = (int64_t *)b_msrc.ensure(8 * E), *md = (int64_t *)b_mdst.ensure(8 * E);
        k_bb_map<<<grid_for(E, 256, 8192), 256, 0, s>>>(perm, dsrc, ddst, E, ms, md);
        GS_HIP(hipGetLastError());
        dsrc = ms;
        ddst = md;
    }
    R.dsrc = dsrc;
    R.ddst = ddst;
    R.osrc = osrc;
    R.odst = odst;
    R.dw = (const double *)to_device(c, b_w, w, sizeof(double) * E, loc);
    R.misc = (unsigned long long *)b_misc.ensure(64);
    GS_HIP(hipMemsetAsync(R.misc, 0, 64, s));
    R.state = (uint8_t *)b_state.ensure(E ? E : 1);
    if (E) GS_HIP(hipMemsetAsync(R.state, 0, E, s));
    R.why = nullptr;
    R.why_E = 0;
    if (R.why_on) {
        R.why = (uint8_t *)c->buf("bb_why").ensure(E ? E : 1);
        if (E) GS_HIP(hipMemsetAsync(R.why, 0, E, s));
        R.why_E = E;
    }
    R.tall = prof_begin(c);
    if (E > 0) {
        hipEvent_t t0 = prof_begin(c);  // ended as "bb_build" below (no leak at E = 0)
        int64_t gnnz = 0;
        bb_build_graph(c, n, E, dsrc, ddst, osrc, odst, R.dw, R.misc, R.gp, R.gi, R.gw, &R.wmed, &gnnz);
        // columns grouped by source row (stable: radix sort is stable)
        uint64_t *okeys = (uint64_t *)b_okeys.ensure(8 * E);
        R.order = (int64_t *)b_order.ensure(8 * E);
        R.optr = (int64_t *)b_optr.ensure(8 * (n + 1));
        k_bb_srckeys<<<grid_for(E, 256, 8192), 256, 0, s>>>(dsrc, E, okeys, R.order);
        sort_pairs_u64_i64(c, okeys, R.order, E, bits_for_bb((uint64_t)n));
        k_bb_rowptr<<<grid_for(n + 1, 256, 8192), 256, 0, s>>>(okeys, E, 1, n, R.optr);
        prof_end(c, t0, "bb_build", 0.0);
        hipEvent_t tp = prof_begin(c);
        // landmark certificates (GSPARSE_BB_LANDMARKS = K, 0 = off; large graphs: 48 --
        // with the reverse-column decisions the searches are what the certificates
        // leave, RMAT-18 711 vs 725 ms at 16; 0: 2.17 s)
        int K = n > 65536 ? 48 : 16;
        if (const char *e = getenv("GSPARSE_BB_LANDMARKS")) K = atoi(e) < 0 ? 0 : atoi(e);
        if (K > n) K = (int)n;
        R.K = K;
        if (K > 0) {
            // landmarks: the K highest-degree nodes of G (ties: the lower id), on the device
            uint64_t *dk = (uint64_t *)c->buf("bb_lmkeys").ensure(8 * n);
            int64_t *di = (int64_t *)c->buf("bb_lmord").ensure(8 * n);
            k_bb_degkeys<<<grid_for(n, 256, 8192), 256, 0, s>>>(R.gp, n, dk, di);
            sort_pairs_u64_i64(c, dk, di, n, 64);
            int32_t *dlm = (int32_t *)b_lm.ensure(4 * K);
            k_bb_first_ids<<<(unsigned)((K + 255) / 256), 256, 0, s>>>(di, K, dlm);
            R.D = (double *)b_land.ensure(8 * (size_t)K * n);
            k_bb_fill_u64<<<grid_for((int64_t)K * n, 256, 65536), 256, 0, s>>>(
                (unsigned long long *)R.D, (int64_t)K * n, kInfBits);
            R.lcomp = (int32_t *)b_lcomp.ensure(4 * K);
            GS_HIP(hipMemsetAsync(R.lcomp, 0, 4 * K, s));
            const int mine = (K - lpart + lparts - 1) / lparts;  // landmarks l = lpart (mod lparts)
            // large graphs: the searches spread over the GPU, one launch per round
            // (k_lm_round; GSPARSE_BB_LMCOOP=0: one workgroup per landmark)
            bool coop = n > 65536 && n < ((int64_t)1 << 31);
            if (const char *e = getenv("GSPARSE_BB_LMCOOP")) coop = coop && atoi(e) != 0;
            if (mine > 0 && coop) {
                const int64_t cap = n + gnnz / kLmChunk + 64;  // items of one round, at most
                uint64_t *items = (uint64_t *)c->buf("bb_lmitems").ensure(16 * (size_t)mine * cap);
                uint32_t *stamp = (uint32_t *)c->buf("bb_lmstamp").ensure(4 * (size_t)mine * n);
                int32_t *cnt = (int32_t *)c->buf("bb_lmcnt").ensure(16 * (size_t)mine);
                unsigned long long *tot = R.misc + 6;
                GS_HIP(hipMemsetAsync(stamp, 0, 4 * (size_t)mine * n, s));
                k_lm_init<<<(unsigned)mine, 256, 0, s>>>(R.gp, dlm, K, lpart, lparts, mine, cap,
                                                         (unsigned long long *)R.D, items, cnt);
                // workgroups per landmark: about two 512-thread workgroups per CU in all
                int W = (512 + mine - 1) / mine;
                if (const char *e = getenv("GSPARSE_BB_LMW")) W = atoi(e);
                W = std::max(1, std::min(W, 256));
                int r = 0;
                while (r < kBbLandmarkRounds) {
                    k_lm_round<512><<<(unsigned)(mine * W), 512, 0, s>>>(
                        R.gp, R.gi, R.gw, n, K, lpart, lparts, W, r, cap, (unsigned long long *)R.D,
                        items, stamp, cnt);
                    ++r;
                    // every 8 rounds: stop once no landmark has a frontier
                    if (r % 8 == 0 && r < kBbLandmarkRounds) {
                        GS_HIP(hipMemsetAsync(tot, 0, 8, s));
                        k_lm_count<<<1, 256, 0, s>>>(cnt, mine, r, lpart, lparts, tot, R.lcomp, 0);
                        unsigned long long ht = 0;
                        GS_HIP(hipMemcpyAsync(&ht, tot, 8, hipMemcpyDeviceToHost, s));
                        GS_HIP(hipStreamSynchronize(s));
                        if (ht == 0) break;
                    }
                }
                GS_HIP(hipMemsetAsync(tot, 0, 8, s));
                k_lm_count<<<1, 256, 0, s>>>(cnt, mine, r, lpart, lparts, tot, R.lcomp, 1);
                GS_HIP(hipGetLastError());
                if (getenv("GSPARSE_BB_DEBUG"))
                    fprintf(stderr, "[backbone] landmarks %d of %d: %d rounds, %d workgroups each\n", mine, K, r, W);
            } else if (mine > 0) {
                unsigned long long *ldist = (unsigned long long *)b_dist.ensure(8 * (size_t)mine * n);
                int32_t *lq = (int32_t *)b_qflag.ensure(4 * (size_t)mine * n);
                int32_t *lfr = (int32_t *)b_fr.ensure(8 * (size_t)mine * n);
                int32_t *ltouch = (int32_t *)b_touched.ensure(4 * (size_t)mine * n);
                k_bb_fill_u64<<<grid_for((int64_t)mine * n, 256, 65536), 256, 0, s>>>(
                    ldist, (int64_t)mine * n, kInfBits);
                GS_HIP(hipMemsetAsync(lq, 0, 4 * (size_t)mine * n, s));
                // one workgroup per landmark: 1,024 threads on large graphs (the K searches
                // are the only work in flight then)
                const unsigned lt = n > 65536 ? 1024 : 256;
                k_bb_landmarks<<<(unsigned)mine, lt, 0, s>>>(R.gp, R.gi, R.gw, n, dlm, K, lpart, lparts,
                                                              kBbLandmarkRounds, R.D, R.lcomp, ldist, lq,
                                                              lfr, ltouch);
                GS_HIP(hipGetLastError());
            }
        }
        prof_end(c, tp, "bb_landmarks", 0.0);
    }
    R.begun = true;
}

// every column's (row * n + col) key sorted, its column, and the position of its reverse
// key (the reverse-column decisions of the searches and the pair certificate); once per run
static void bb_keys(gs_ctx *c) {
    BbRun &R = bb_run(c);
    if (R.keys_ready) return;
    hipStream_t s = c->stream;
    const int64_t E = R.E, n = R.n;
    R.skeys = (uint64_t *)c->buf("bb_skeys").ensure(8 * E);
    R.sidx = (int64_t *)c->buf("bb_sidx").ensure(8 * E);
    R.rpos = (int64_t *)c->buf("bb_rpos").ensure(8 * E);
    k_bb_pairkeys<<<grid_for(E, 256, 8192), 256, 0, s>>>(R.dsrc, R.ddst, E, n, R.skeys, R.sidx);
    sort_pairs_u64_i64(c, R.skeys, R.sidx, E, bits_for_bb((uint64_t)n * (uint64_t)n));
    k_bb_revpos<<<grid_for(E, 256, 8192), 256, 0, s>>>(R.dsrc, R.ddst, E, n, R.skeys, R.rpos);
    GS_HIP(hipGetLastError());
    R.keys_ready = true;
}

// the pair certificate's columns in [c0, c1): open, not a self-loop, one of each
// (u, v) / (v, u) pair (the u < v one when both are open)
__global__ void k_bb_pairflag(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                              const uint8_t *__restrict__ state, const int64_t *__restrict__ rpos,
                              const int64_t *__restrict__ sidx, int64_t c0, int64_t c1,
                              int64_t *__restrict__ flag) {
    for (int64_t i = c0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < c1;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[i], v = dst[i];
        int64_t f = 0;
        if (state[i] == 0 && u != v) {
            const int64_t rp = rpos[i];
            f = (u < v || rp < 0 || state[sidx[rp]] != 0) ? 1 : 0;
        }
        flag[i - c0] = f;
    }
}

// lmflag[x] = 1 for the complete landmarks (k_bb_sssp_multi PAIR does not expand them)
__global__ void k_bb_lmflag(const int32_t *__restrict__ lm, const int32_t *__restrict__ lcomp, int K,
                            uint8_t *__restrict__ lmflag) {
    for (int l = threadIdx.x; l < K; l += blockDim.x)
        if (lcomp[l]) lmflag[lm[l]] = 1;
}

__global__ void k_bb_pcompact(const int64_t *__restrict__ flag, const int64_t *__restrict__ pos,
                              int64_t c0, int64_t cnt, int64_t *__restrict__ out) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < cnt;
         j += (int64_t)gridDim.x * blockDim.x)
        if (flag[j]) out[pos[j]] = c0 + j;
}

// witness + certificates of columns [E part / nparts, E (part + 1) / nparts)
static void bb_certify(gs_ctx *c, int part, int nparts) {
    BbRun &R = bb_run(c);
    GS_CHECK(R.begun, GS_ESTATE, "gs_bb_begin first");
    GS_CHECK(nparts >= 1 && 0 <= part && part < nparts, GS_EINVAL, "bad part %d of %d", part, nparts);
    GS_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int64_t E = R.E, c0 = E * part / nparts, c1 = E * (part + 1) / nparts;
    hipEvent_t tp = prof_begin(c);
    if (c1 > c0) {
        // the certificates first (landmarks, local bounds: O(K) / O(log d) per column), then
        // the 2-hop witnesses of the columns still open -- a merge of both endpoints'
        // lists, which the hub-hub columns the landmark labels decide made the dearest
        // local bounds (k_bb_certify; GSPARSE_BB_LOCALLB=0: off)
        bool local = true;
        if (const char *e = getenv("GSPARSE_BB_LOCALLB")) local = atoi(e) != 0;
        double *mw = nullptr, *aw = nullptr;
        int32_t *ma = nullptr, *aa = nullptr;
        const double mrg = std::max(1e-8, 8.0 * (double)R.n * 0x1p-53);
        if (local && R.n > 0) {
            mw = (double *)c->buf("bb_minw").ensure(16 * (size_t)R.n);
            ma = (int32_t *)c->buf("bb_mina").ensure(4 * (size_t)R.n);
            k_bb_minw<<<grid_for(R.n * 64, 256, 16384), 256, 0, s>>>(R.gp, R.gi, R.gw, R.n, mw, ma);
            aw = (double *)c->buf("bb_minw2").ensure(16 * (size_t)R.n);
            aa = (int32_t *)c->buf("bb_mina2").ensure(4 * (size_t)R.n);
            k_bb_minw2<<<grid_for(R.n * 64, 256, 16384), 256, 0, s>>>(R.gp, R.gi, R.gw, R.n, mw, ma, aw, aa);
        }
        if (R.K > 0 || local) {
            k_bb_certify<<<grid_for(c1 - c0, 256, 8192), 256, 0, s>>>(R.dsrc, R.ddst, R.dw, c0, c1, R.gp,
                                                                       R.gi, R.gw, R.D, R.lcomp, R.K,
                                                                       R.eps, mrg, mw, ma, R.pair_part,
                                                                       R.pair_nparts, R.state, R.why);
        }
        k_bb_witness<<<grid_for(c1 - c0, 256, 8192), 256, 0, s>>>(
            R.dsrc, R.ddst, R.dw, c0, c1, R.gp, R.gi, R.gw, R.eps, R.pair_part, R.pair_nparts, mw, ma,
            aw, aa, mrg, R.state, R.why);
        // the meet-in-the-middle certificate of the columns still open (k_bb_sssp_multi
        // PAIR: both ends searched to half the column's weight; GSPARSE_BB_MITM=1: on).
        // It needs the local bounds' direct-edge rule, so it runs only with them.  Off by
        // default: on R-MAT-18 it decides all but 202 of the 204 k open columns, but the
        // balls of radius ~9 around their (hub-adjacent) ends already hold ~0.28 E
        // relaxations each -- 1.2·10¹¹ for the 102 k pairs, 3.3 s against 0.38 s for the
        // searches it replaces (profiles/r05z10_*).
        bool mitm = false;
        if (const char *e = getenv("GSPARSE_BB_MITM")) mitm = local && atoi(e) != 0;
        if (mitm) {
            hipEvent_t tq = prof_begin(c);
            bb_keys(c);
            const int64_t nc = c1 - c0;
            int64_t *pf = (int64_t *)c->buf("bb_pflag").ensure(8 * (nc + 1));
            int64_t *pp = (int64_t *)c->buf("bb_ppos").ensure(8 * (nc + 1));
            k_bb_pairflag<<<grid_for(nc, 256, 8192), 256, 0, s>>>(R.dsrc, R.ddst, R.state, R.rpos, R.sidx, c0,
                                                                   c1, pf);
            exclusive_scan_i64(c, pf, pp, nc);
            int64_t lastp = 0, lastf = 0;
            GS_HIP(hipMemcpyAsync(&lastp, pp + nc - 1, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipMemcpyAsync(&lastf, pf + nc - 1, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            const int64_t np = lastp + lastf;
            if (getenv("GSPARSE_BB_DEBUG"))
                fprintf(stderr, "[backbone] pair certificate: %lld open pairs\n", (long long)np);
            if (np > 0) {
                int64_t *plist = (int64_t *)c->buf("bb_plist").ensure(8 * np);
                k_bb_pcompact<<<grid_for(nc, 256, 8192), 256, 0, s>>>(pf, pp, c0, nc, plist);
                int64_t P = 512;
                if (const char *e = getenv("GSPARSE_BB_MITM_SLABS")) P = atoi(e) > 0 ? atoi(e) : P;
                P = std::min<int64_t>(P, np);
                const int64_t cap = (int64_t)(48e9 / (44.0 * (double)R.n));  // slab bytes per node: 2 x 8 + 28
                if (P > cap) P = std::max<int64_t>(cap, 1);
                const size_t dbytes = 16 * (size_t)P * R.n, qbytes = 4 * (size_t)P * R.n;
                auto *dist = (unsigned long long *)c->buf("bb_dist").ensure(dbytes);
                auto *qm = (uint32_t *)c->buf("bb_qflag").ensure(qbytes);
                auto *fr = (int32_t *)c->buf("bb_fr").ensure(8 * (size_t)P * R.n);
                auto *fm = (uint32_t *)c->buf("bb_fmask").ensure(4 * (size_t)P * R.n);
                auto *tch = (int32_t *)c->buf("bb_touched").ensure(4 * (size_t)P * R.n);
                auto *farl = (int32_t *)c->buf("bb_far").ensure(8 * (size_t)P * R.n);
                if (R.dist_ok != (void *)dist || R.dist_ok_bytes < dbytes) {
                    k_bb_fill_u64<<<grid_for((int64_t)(dbytes / 8), 256, 65536), 256, 0, s>>>(
                        dist, (int64_t)(dbytes / 8), kInfBits);
                    R.dist_ok = dist;
                    R.dist_ok_bytes = dbytes;
                }
                if (R.q_ok != (void *)qm || R.q_ok_bytes < qbytes) {
                    GS_HIP(hipMemsetAsync(qm, 0, qbytes, s));
                    R.q_ok = qm;
                    R.q_ok_bytes = qbytes;
                }
                double nfs = 2.0;
                if (const char *e = getenv("GSPARSE_BB_NEARFAR")) nfs = atof(e);
                const double delta = nfs > 0.0 && R.wmed > 0.0 ? nfs * R.wmed : 0.0;
                unsigned long long *bnext = R.misc + 2;
                GS_HIP(hipMemsetAsync(bnext, 0, 8, s));
                // complete landmarks blocked (GSPARSE_BB_MITM_LM=0: expanded like any node)
                uint8_t *lmf = nullptr;
                bool lmb = R.K > 0;
                if (const char *e = getenv("GSPARSE_BB_MITM_LM")) lmb = lmb && atoi(e) != 0;
                if (lmb) {
                    lmf = (uint8_t *)c->buf("bb_lmflag").ensure((size_t)R.n);
                    GS_HIP(hipMemsetAsync(lmf, 0, (size_t)R.n, s));
                    k_bb_lmflag<<<1, 64, 0, s>>>((const int32_t *)c->buf("bb_lm").ptr, R.lcomp, R.K, lmf);
                }
                // GSPARSE_BB_TRACE: as bb_search's, one line per launch ("pairs": true)
                const char *tpath = getenv("GSPARSE_BB_TRACE");
                unsigned long long *trace = nullptr;
                if (tpath) {
                    trace = (unsigned long long *)c->buf("bb_trace").ensure(48 * (size_t)np);
                    GS_HIP(hipMemsetAsync(trace, 0, 48 * (size_t)np, s));
                }
                k_bb_sssp_multi<512, 2, true><<<(unsigned)P, 512, 0, s>>>(
                    R.gp, R.gi, R.gw, R.n, plist, np, R.optr, R.order, R.dsrc, R.ddst, R.dw, R.eps, R.state,
                    dist, qm, fr, fm, tch, farl, delta, 0, R.skeys, R.sidx, R.rpos, R.E, mrg, 0, 0, np, 0, 1,
                    bnext, R.misc + 1, trace, R.why, lmf, R.D, R.lcomp, R.K);
                GS_HIP(hipGetLastError());
                if (tpath) {
                    std::vector<unsigned long long> h(6 * (size_t)np);
                    GS_HIP(hipMemcpyAsync(h.data(), trace, 48 * (size_t)np, hipMemcpyDeviceToHost, s));
                    GS_HIP(hipStreamSynchronize(s));
                    if (FILE *f = fopen(tpath, "a")) {
                        fprintf(f, "{\"pairs\": true, \"part\": %d, \"nparts\": %d, \"b0\": 0, \"b1\": %lld, \"S\": 2, \"grid\": %lld, \"rec\": [",
                                part, nparts, (long long)np, (long long)P);
                        for (int64_t i = 0; i < np; ++i) {
                            double bm;
                            memcpy(&bm, &h[6 * i + 3], 8);
                            fprintf(f, "%s[%llu, %llu, %llu, %.9g, %llu, %llu]", i ? ", " : "", h[6 * i], h[6 * i + 1],
                                    h[6 * i + 2], bm, h[6 * i + 4], h[6 * i + 5]);
                        }
                        fprintf(f, "]}\n");
                        fclose(f);
                    }
                }
            }
            prof_end(c, tq, "bb_pairs", 0.0);
        }
        GS_HIP(hipGetLastError());
    }
    prof_end(c, tp, "bb_certify", 0.0);
    R.certified = true;
}

// the sources with open columns, in node order (the same list on every rank), and the
// search geometry
static void bb_plan(gs_ctx *c) {
    BbRun &R = bb_run(c);
    GS_CHECK(R.certified, GS_ESTATE, "gs_bb_certify first");
    GS_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int64_t n = R.n, E = R.E;
    R.nsrc = R.nbatch = 0;
    hipEvent_t tp = prof_begin(c);
    if (E > 0) {
        int64_t *flag = (int64_t *)c->buf("bb_flag").ensure(8 * (n + 1));
        int64_t *pos = (int64_t *)c->buf("bb_pos").ensure(8 * (n + 1));
        hipEvent_t tq = prof_begin(c);
        GS_HIP(hipMemsetAsync(flag, 0, 8 * (n + 1), s));
        k_bb_need<<<grid_for(E, 256, 8192), 256, 0, s>>>(R.dsrc, R.state, E, flag);
        exclusive_scan_i64(c, flag, pos, n);
        int64_t lastp = 0, lastf = 0;
        if (n) {
            GS_HIP(hipMemcpyAsync(&lastp, pos + n - 1, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipMemcpyAsync(&lastf, flag + n - 1, 8, hipMemcpyDeviceToHost, s));
        }
        GS_HIP(hipStreamSynchronize(s));
        prof_end(c, tq, "bb_plan_need", 0.0);
        R.nsrc = lastp + lastf;
        if (getenv("GSPARSE_BB_DEBUG")) {
            GS_HIP(hipMemsetAsync(R.misc + 3, 0, 8, s));
            k_bb_count0<<<grid_for(E, 256, 4096), 256, 0, s>>>(R.state, E, R.misc + 3);
            unsigned long long open = 0;
            GS_HIP(hipMemcpyAsync(&open, R.misc + 3, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            fprintf(stderr, "[backbone] open before searches=%llu sources=%lld\n", open,
                    (long long)R.nsrc);
        }
        if (R.nsrc > 0) {
            R.sources = (int64_t *)c->buf("bb_sources").ensure(8 * R.nsrc);
            k_bb_compact<<<grid_for(n, 256, 8192), 256, 0, s>>>(flag, pos, n, R.sources);
            // large graphs (big search balls): 512 workgroups of 512 threads, two per CU
            // (RMAT-18 with the final search: 650 vs 692 ms for 256 x 1,024; round 1's
            // plain search preferred 256 x 1,024); small ones (many short searches):
            // 1,024 workgroups of 256 (Roman: 2.2 vs 3.0 ms)
            const bool big = n > 65536;
            // a rank of 8 or more (staged form) has few batches per workgroup and waits on
            // single searches: 2 sources per workgroup of 1,024 threads, 256 workgroups
            // (RMAT-18 at N = 8: 120.5 ms per rank vs 131.5 ms with 8 sources x 512
            // threads; at N = 4 the latter wins, 188.8 vs 204.9 ms; tools/bb_stage_probe.py,
            // profiles/r05t_*)
            const bool wide = big && R.nranks >= 8;
            int64_t maxslabs = big ? (wide ? 256 : 512) : 1024;
            if (const char *e = getenv("GSPARSE_BB_SLABS")) maxslabs = atoi(e) > 0 ? atoi(e) : maxslabs;
            // sources searched together per workgroup (k_bb_sssp_multi), 1 = alone: on
            // large graphs 16 on one GPU (RMAT-18 with the local-bound certificates: 455.9
            // vs 475.8 ms with 8, which keep the near-far order), 8 per rank of 2 to 7 (N = 4:
            // 188.8 ms; 16: 219.7); alone on small ones (Roman: 2.30 ms vs 2.45 ms with 8)
            int S = big ? (wide ? 2 : R.nranks == 1 ? 16 : 8) : 1;
            if (const char *e = getenv("GSPARSE_BB_MULTI")) {
                const int v = atoi(e);
                S = v >= 16 ? 16 : v >= 8 ? 8 : v >= 4 ? 4 : v >= 2 ? 2 : 1;
            }
            R.S = S;
            R.nbatch = (R.nsrc + S - 1) / S;
            int64_t slabs = R.nbatch < maxslabs ? R.nbatch : maxslabs;
            // keep the working set of all slabs under ~48 GB (of 288)
            const double per = S == 1 ? 24.0 : 8.0 * S + 28.0;
            int64_t cap = (int64_t)(48e9 / (per * (double)(n ? n : 1)));
            if (cap < 1) cap = 1;
            if (slabs > cap) slabs = cap;
            R.slabs = slabs;
            hipEvent_t tf = prof_begin(c);
            const size_t dbytes = 8 * (size_t)S * slabs * n, qbytes = 4 * (size_t)slabs * n;
            R.dist = (unsigned long long *)c->buf("bb_dist").ensure(dbytes);
            R.qflag = (int32_t *)c->buf("bb_qflag").ensure(qbytes);
            R.fr = (int32_t *)c->buf("bb_fr").ensure(8 * slabs * n);
            R.touched = (int32_t *)c->buf("bb_touched").ensure(4 * slabs * n);
            // (RMAT-18, 16 sources x 512 slabs: 17 GB, 3.2 ms per prune when filled each time)
            const bool refill = getenv("GSPARSE_BB_REFILL") != nullptr;
            if (refill || R.dist_ok != (void *)R.dist || R.dist_ok_bytes < dbytes) {
                k_bb_fill_u64<<<grid_for((int64_t)S * slabs * n, 256, 65536), 256, 0, s>>>(
                    R.dist, (int64_t)S * slabs * n, kInfBits);
                R.dist_ok = R.dist;
                R.dist_ok_bytes = dbytes;
            }
            if (refill || R.q_ok != (void *)R.qflag || R.q_ok_bytes < qbytes) {
                GS_HIP(hipMemsetAsync(R.qflag, 0, qbytes, s));
                R.q_ok = R.qflag;
                R.q_ok_bytes = qbytes;
            }
            prof_end(c, tf, "bb_plan_fill", 0.0);
            R.bt = big ? (wide ? 1024 : 512) : 256;
            if (const char *e = getenv("GSPARSE_BB_THREADS")) R.bt = atoi(e) == 1024 ? 1024 : atoi(e) == 512 ? 512 : 256;
            if (S > 1) {
                R.fm = (uint32_t *)c->buf("bb_fmask").ensure(4 * slabs * n);
                // reverse-column decisions after every search (GSPARSE_BB_CROSS=0: off)
                R.cross = 1;
                if (const char *e = getenv("GSPARSE_BB_CROSS")) R.cross = atoi(e) != 0;
                hipEvent_t tc = prof_begin(c);
                if (R.cross) bb_keys(c);
                prof_end(c, tc, "bb_plan_cross", 0.0);
                // sources by ascending column count (the batches from the last): the
                // short searches first, so their reverse-column decisions close most of
                // the hubs' targets before the hubs search (RMAT-18 1.63 -> 0.83 s;
                // GSPARSE_BB_ORDER=desc: hubs first)
                R.rev = 1;
                if (const char *e = getenv("GSPARSE_BB_ORDER")) R.rev = strcmp(e, "desc") != 0;
                // batches from a global counter (misc + 2); GSPARSE_BB_DYNAMIC=0: static striding
                R.dynamic = true;
                if (const char *e = getenv("GSPARSE_BB_DYNAMIC")) R.dynamic = atoi(e) != 0;
                R.farl = (int32_t *)c->buf("bb_far").ensure(8 * slabs * n);
                // near-far step: twice the median edge weight (GSPARSE_BB_NEARFAR = the
                // factor, 0 = plain frontier order; RMAT-18: 1 / 2 / 4 -> 687 / 692 / 700 ms
                // at 256 x 1,024 threads, 0 -> 723 ms)
                double nfs = 2.0;
                if (const char *e = getenv("GSPARSE_BB_NEARFAR")) nfs = atof(e);
                R.delta = nfs > 0.0 && R.wmed > 0.0 ? nfs * R.wmed : 0.0;
            }
            GS_HIP(hipGetLastError());
        }
    }
    prof_end(c, tp, "bb_plan", 0.0);
    R.planned = true;
}

// search batches [b0, b1) of the processing order, this part's every nparts-th one
static void bb_search(gs_ctx *c, int64_t b0, int64_t b1, int part, int nparts) {
    BbRun &R = bb_run(c);
    GS_CHECK(R.planned, GS_ESTATE, "gs_bb_plan first");
    GS_CHECK(nparts >= 1 && 0 <= part && part < nparts, GS_EINVAL, "bad part %d of %d", part, nparts);
    GS_CHECK(0 <= b0 && b0 <= b1 && b1 <= R.nbatch, GS_EINVAL, "batches [%lld, %lld) outside [0, %lld)",
             (long long)b0, (long long)b1, (long long)R.nbatch);
    GS_HIP(hipSetDevice(c->device));
    if (b1 - b0 <= part) return;  // none of this part's
    hipStream_t s = c->stream;
    const int64_t mine = (b1 - b0 - part + nparts - 1) / nparts;
    const unsigned grid = (unsigned)std::min<int64_t>(R.slabs, mine);
    hipEvent_t tp = prof_begin(c);
    if (R.S == 1) {
        auto kfn = R.bt == 1024 ? k_bb_sssp<1024> : R.bt == 512 ? k_bb_sssp<512> : k_bb_sssp<256>;
        kfn<<<grid, R.bt, 0, s>>>(R.gp, R.gi, R.gw, R.n, R.sources, R.nsrc, R.optr, R.order, R.ddst,
                                  R.dw, R.eps, R.state, R.dist, R.qflag, R.fr, R.touched, b0, b1, part,
                                  nparts, R.misc + 1, R.why);
    } else {
        unsigned long long *bnext = R.dynamic ? R.misc + 2 : nullptr;
        if (bnext) GS_HIP(hipMemsetAsync(bnext, 0, 8, s));
        const double mrg = std::max(1e-8, 8.0 * (double)R.n * 0x1p-53);
        auto *qm = (uint32_t *)R.qflag;
        // GSPARSE_BB_TRACE=file: each batch's start / end (constant clock, 100 MHz) and
        // workgroup, one JSON line per launch appended to the file (waits for the launch)
        const char *tpath = getenv("GSPARSE_BB_TRACE");
        unsigned long long *trace = nullptr;
        if (tpath) {
            trace = (unsigned long long *)c->buf("bb_trace").ensure(48 * (size_t)mine);
            GS_HIP(hipMemsetAsync(trace, 0, 48 * (size_t)mine, s));
        }
#define GS_BBM(NT_, S_)                                                                          \
    k_bb_sssp_multi<NT_, S_><<<grid, NT_, 0, s>>>(R.gp, R.gi, R.gw, R.n, R.sources, R.nsrc, R.optr, \
                                                   R.order, R.dsrc, R.ddst, R.dw, R.eps, R.state, R.dist,  \
                                                   qm, R.fr, R.fm, R.touched, R.farl, R.delta,     \
                                                   R.cross, R.skeys, R.sidx, R.rpos, R.E, mrg,     \
                                                   R.rev, b0, b1, part, nparts, bnext, R.misc + 1, \
                                                   trace, R.why)
        const int S = R.S;
        if (R.bt == 1024) {
            if (S == 2) GS_BBM(1024, 2); else if (S == 4) GS_BBM(1024, 4);
            else if (S == 8) GS_BBM(1024, 8); else GS_BBM(1024, 16);
        } else if (R.bt == 512) {
            if (S == 2) GS_BBM(512, 2); else if (S == 4) GS_BBM(512, 4);
            else if (S == 8) GS_BBM(512, 8); else GS_BBM(512, 16);
        } else {
            if (S == 2) GS_BBM(256, 2); else if (S == 4) GS_BBM(256, 4);
            else if (S == 8) GS_BBM(256, 8); else GS_BBM(256, 16);
        }
#undef GS_BBM
        if (tpath) {
            std::vector<unsigned long long> h(6 * (size_t)mine);
            GS_HIP(hipMemcpyAsync(h.data(), trace, 48 * (size_t)mine, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            if (FILE *f = fopen(tpath, "a")) {
                fprintf(f, "{\"part\": %d, \"nparts\": %d, \"b0\": %lld, \"b1\": %lld, \"S\": %d, \"grid\": %u, \"rec\": [",
                        part, nparts, (long long)b0, (long long)b1, R.S, grid);
                for (int64_t i = 0; i < mine; ++i) {
                    double bm;
                    memcpy(&bm, &h[6 * i + 3], 8);
                    fprintf(f, "%s[%llu, %llu, %llu, %.9g, %llu, %llu]", i ? ", " : "", h[6 * i], h[6 * i + 1],
                            h[6 * i + 2], bm, h[6 * i + 4], h[6 * i + 5]);
                }
                fprintf(f, "]}\n");
                fclose(f);
            }
        }
    }
    GS_HIP(hipGetLastError());
    prof_end(c, tp, "bb_search", 0.0);
}

static void bb_finish(gs_ctx *c, uint8_t *keep, int keep_loc, int64_t *n_relax) {
    BbRun &R = bb_run(c);
    GS_CHECK(R.certified, GS_ESTATE, "gs_bb_certify first");
    GS_CHECK(R.E == 0 || keep, GS_EINVAL, "null keep array");
    GS_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const int64_t E = R.E;
    uint8_t *dkeep = (uint8_t *)out_device(c, c->buf("bb_keep"), keep, E ? E : 1, keep_loc);
    int64_t relax = 0;
    if (E > 0) {
        k_bb_keep<<<grid_for(E, 256, 8192), 256, 0, s>>>(R.state, R.dsrc, R.ddst, E, R.pair_part,
                                                       R.pair_nparts, dkeep);
        GS_HIP(hipGetLastError());
        unsigned long long hr = 0;
        GS_HIP(hipMemcpyAsync(&hr, R.misc + 1, 8, hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        relax = (int64_t)hr;
    }
    prof_end(c, R.tall, "metric_backbone", 12.0 * (double)relax + 9.0 * (double)E);
    R.tall = nullptr;
    finish_out(c, keep, dkeep, E, keep_loc);
    if (n_relax) *n_relax = relax;
    R.begun = R.certified = R.planned = false;
}

extern "C" int gs_metric_backbone_part(gs_ctx *c, int64_t n, int64_t E, const int64_t *src,
                                       const int64_t *dst, const double *w, int64_t nw, int loc,
                                       double eps, int part, int nparts, uint8_t *keep,
                                       int keep_loc, int64_t *n_relax) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(E == 0 || keep, GS_EINVAL, "null column/weight/keep array");
        bb_begin(c, n, E, src, dst, w, nw, loc, eps, 0, 1, part, nparts);
        bb_certify(c, 0, 1);
        bb_plan(c);
        bb_search(c, 0, bb_run(c).nbatch, 0, 1);
        bb_finish(c, keep, keep_loc, n_relax);
    });
}

extern "C" int gs_metric_backbone(gs_ctx *c, int64_t n, int64_t E, const int64_t *src,
                                  const int64_t *dst, const double *w, int64_t nw, int loc,
                                  double eps, uint8_t *keep, int keep_loc, int64_t *n_relax) {
    return gs_metric_backbone_part(c, n, E, src, dst, w, nw, loc, eps, 0, 1, keep, keep_loc,
                                   n_relax);
}

extern "C" int gs_bb_begin(gs_ctx *c, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                           const double *w, int64_t nw, int loc, double eps, int part, int nparts,
                           int32_t *n_landmarks) {
    return guard([&] {
        bb_begin(c, n, E, src, dst, w, nw, loc, eps, part, nparts, 0, 1);
        if (n_landmarks) *n_landmarks = bb_run(c).K;
    });
}

extern "C" int gs_bb_landmarks_io(gs_ctx *c, double *D, int32_t *complete, int loc, int dir) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        BbRun &R = bb_run(c);
        GS_CHECK(R.begun, GS_ESTATE, "gs_bb_begin first");
        GS_CHECK(dir == 0 || dir == 1, GS_EINVAL, "dir must be 0 (out) or 1 (in)");
        if (R.K == 0 || R.E == 0) return;
        GS_CHECK(D && complete, GS_EINVAL, "null landmark buffers");
        GS_HIP(hipSetDevice(c->device));
        const size_t nd = 8 * (size_t)R.K * R.n, nc = 4 * (size_t)R.K;
        const hipMemcpyKind k = loc == GS_DEVICE ? hipMemcpyDeviceToDevice
                                : dir == 0 ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
        if (dir == 0) {
            GS_HIP(hipMemcpyAsync(D, R.D, nd, k, c->stream));
            GS_HIP(hipMemcpyAsync(complete, R.lcomp, nc, k, c->stream));
        } else {
            GS_HIP(hipMemcpyAsync(R.D, D, nd, k, c->stream));
            GS_HIP(hipMemcpyAsync(R.lcomp, complete, nc, k, c->stream));
        }
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

extern "C" int gs_bb_certify(gs_ctx *c, int part, int nparts) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        bb_certify(c, part, nparts);
    });
}

extern "C" int gs_bb_state_io(gs_ctx *c, uint8_t *state, int loc, int dir) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        BbRun &R = bb_run(c);
        GS_CHECK(R.begun, GS_ESTATE, "gs_bb_begin first");
        GS_CHECK(dir == 0 || dir == 1, GS_EINVAL, "dir must be 0 (out) or 1 (in)");
        if (R.E == 0) return;
        GS_CHECK(state, GS_EINVAL, "null state buffer");
        GS_HIP(hipSetDevice(c->device));
        const hipMemcpyKind k = loc == GS_DEVICE ? hipMemcpyDeviceToDevice
                                : dir == 0 ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
        if (dir == 0) GS_HIP(hipMemcpyAsync(state, R.state, R.E, k, c->stream));
        else GS_HIP(hipMemcpyAsync(R.state, state, R.E, k, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

extern "C" int gs_bb_plan(gs_ctx *c, int64_t *nbatch) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        bb_plan(c);
        if (nbatch) *nbatch = bb_run(c).nbatch;
    });
}

extern "C" int gs_bb_search(gs_ctx *c, int64_t b0, int64_t b1, int part, int nparts) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        bb_search(c, b0, b1, part, nparts);
    });
}

extern "C" int gs_bb_finish(gs_ctx *c, uint8_t *keep, int keep_loc, int64_t *n_relax) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        bb_finish(c, keep, keep_loc, n_relax);
    });
}

__global__ void k_bb_why_hist(const uint8_t *__restrict__ why, int64_t E,
                              unsigned long long *__restrict__ cnt) {
    __shared__ unsigned int h[kWhyClasses];
    for (int k = threadIdx.x; k < kWhyClasses; k += blockDim.x) h[k] = 0;
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t k = why[i];
        atomicAdd(&h[k < kWhyClasses ? k : 0], 1u);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kWhyClasses; k += blockDim.x)
        if (h[k]) atomicAdd(&cnt[k], (unsigned long long)h[k]);
}

extern "C" int gs_bb_classes(gs_ctx *c, int on) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        bb_run(c).why_on = on != 0;
    });
}

extern "C" int gs_bb_class_counts(gs_ctx *c, int64_t *counts, int ncounts, uint8_t *why, int64_t nwhy,
                                  int why_loc, int64_t *n_columns) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(counts && ncounts >= (int)kWhyClasses, GS_EINVAL, "counts needs %d entries", (int)kWhyClasses);
        BbRun &R = bb_run(c);
        GS_CHECK(R.why_on && R.why, GS_ESTATE, "gs_bb_classes(ctx, 1) before the backbone run");
        GS_CHECK(!why || nwhy >= R.why_E, GS_EINDEX, "why holds %lld bytes, the run has %lld columns",
                 (long long)nwhy, (long long)R.why_E);
        if (n_columns) *n_columns = R.why_E;
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        auto *d = (unsigned long long *)c->buf("bb_whycnt").ensure(8 * kWhyClasses);
        GS_HIP(hipMemsetAsync(d, 0, 8 * kWhyClasses, s));
        if (R.why_E > 0) k_bb_why_hist<<<grid_for(R.why_E, 256, 2048), 256, 0, s>>>(R.why, R.why_E, d);
        GS_HIP(hipGetLastError());
        unsigned long long h[kWhyClasses];
        GS_HIP(hipMemcpyAsync(h, d, 8 * kWhyClasses, hipMemcpyDeviceToHost, s));
        if (why && R.why_E > 0)
            GS_HIP(hipMemcpyAsync(why, R.why, R.why_E,
                                  why_loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        for (int k = 0; k < ncounts; ++k) counts[k] = k < (int)kWhyClasses ? (int64_t)h[k] : 0;
    });
}

extern "C" int gs_pair_distances(gs_ctx *c, int64_t n, int64_t E, const int64_t *src,
                                 const int64_t *dst, const double *w, int64_t nw, int loc,
                                 int64_t nq, const int64_t *qs, const int64_t *qt, double *out) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(!w || nw >= E, GS_EINDEX, "index %lld is out of bounds for axis 0 with size %lld",
                 (long long)nw, (long long)nw);
        GS_CHECK(n >= 0 && E >= 0 && nq >= 0, GS_EINVAL, "negative n/E/nq");
        GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31");
        GS_CHECK(nq == 0 || (qs && qt && out), GS_EINVAL, "null query arrays");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        if (nq == 0) return;
        // queries (host) grouped by source, in a stable order
        std::vector<int64_t> ord((size_t)nq);
        for (int64_t q = 0; q < nq; ++q) {
            GS_CHECK(qs[q] >= 0 && qs[q] < n && qt[q] >= 0 && qt[q] < n, GS_EINVAL,
                     "query %lld out of range [0, %lld)", (long long)q, (long long)n);
            ord[(size_t)q] = q;
        }
        std::stable_sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) { return qs[a] < qs[b]; });
        std::vector<int64_t> srcs, qptr, tq((size_t)nq);
        for (int64_t i = 0; i < nq; ++i) {
            const int64_t q = ord[(size_t)i];
            if (srcs.empty() || srcs.back() != qs[q]) {
                srcs.push_back(qs[q]);
                qptr.push_back(i);
            }
            tq[(size_t)i] = qt[q];
        }
        qptr.push_back(nq);
        const int64_t nsrc = (int64_t)srcs.size();
        std::vector<double> res((size_t)nq, __builtin_inf());
        if (E > 0) {
            const int64_t *dsrc = (const int64_t *)to_device(c, c->buf("bp_src"), src, 8 * E, loc);
            const int64_t *ddst = (const int64_t *)to_device(c, c->buf("bp_dst"), dst, 8 * E, loc);
            const double *dw;
            if (w) {
                dw = (const double *)to_device(c, c->buf("bp_w"), w, 8 * E, loc);
            } else {  // unweighted: hop counts (sums of 1.0 are exact)
                double *d1 = (double *)c->buf("bp_w").ensure(8 * E);
                k_bb_fill_u64<<<grid_for(E, 256, 8192), 256, 0, s>>>(
                    (unsigned long long *)d1, E, 0x3ff0000000000000ull);  // 1.0
                dw = d1;
            }
            auto *misc = (unsigned long long *)c->buf("bp_misc").ensure(64);
            GS_HIP(hipMemsetAsync(misc, 0, 64, s));
            int64_t *gp;
            int32_t *gi;
            double *gw;
            bb_build_graph(c, n, E, dsrc, ddst, dsrc, ddst, dw, misc, gp, gi, gw);
            int64_t *d_src = (int64_t *)c->buf("bp_srcs").ensure(8 * nsrc);
            int64_t *d_ptr = (int64_t *)c->buf("bp_qptr").ensure(8 * (nsrc + 1));
            int64_t *d_tq = (int64_t *)c->buf("bp_tq").ensure(8 * nq);
            double *d_out = (double *)c->buf("bp_out").ensure(8 * nq);
            GS_HIP(hipMemcpyAsync(d_src, srcs.data(), 8 * nsrc, hipMemcpyHostToDevice, s));
            GS_HIP(hipMemcpyAsync(d_ptr, qptr.data(), 8 * (nsrc + 1), hipMemcpyHostToDevice, s));
            GS_HIP(hipMemcpyAsync(d_tq, tq.data(), 8 * nq, hipMemcpyHostToDevice, s));
            const int64_t slabs = nsrc < 256 ? nsrc : 256;
            auto *dist = (unsigned long long *)c->buf("bb_dist").ensure(8 * slabs * n);
            auto *qflag = (int32_t *)c->buf("bb_qflag").ensure(4 * slabs * n);
            auto *fr = (int32_t *)c->buf("bb_fr").ensure(8 * slabs * n);
            auto *touched = (int32_t *)c->buf("bb_touched").ensure(4 * slabs * n);
            k_bb_fill_u64<<<grid_for(slabs * n, 256, 65536), 256, 0, s>>>(dist, slabs * n, kInfBits);
            GS_HIP(hipMemsetAsync(qflag, 0, 4 * slabs * n, s));
            k_bb_pairs<<<(unsigned)slabs, 256, 0, s>>>(gp, gi, gw, n, d_src, d_ptr, d_tq, nsrc, d_out,
                                                       dist, qflag, fr, touched);
            GS_HIP(hipGetLastError());
            std::vector<double> hout((size_t)nq);
            GS_HIP(hipMemcpyAsync(hout.data(), d_out, 8 * nq, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            for (int64_t i = 0; i < nq; ++i) res[(size_t)ord[(size_t)i]] = hout[(size_t)i];
        }
        for (int64_t q = 0; q < nq; ++q) out[q] = qs[q] == qt[q] ? 0.0 : res[(size_t)q];
    });
}
