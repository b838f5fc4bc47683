// gs_jaccard.hip -- Jaccard (metrics.py:17-64) on symmetric graphs, whole edge set.
//
// For a symmetric graph |out(u) ∩ in(v)| = |N(u) ∩ N(v)| is symmetric in (u, v),
// so each undirected pair is intersected ONCE, at its owner: the endpoint of
// larger degree (ties: smaller id).  The owner row's neighbour set is put in a
// hash table (LDS) or a bitmap (global, for rows too large for LDS) and the
// other endpoint's -- shorter -- list is streamed and probed.  Work is
// sum over pairs of min(d_u, d_v) probes instead of the d_u + d_v of a merge
// (RMAT-22: 1.24e10 vs 2.9e11), and the same value is written to both CSR
// entries (u,v) and (v,u) (rev(e) = tpos[e] on a symmetric graph).
//
// Rows are classed by degree:
//   light (d <= 32): one thread per owned entry, sorted-list merge
//   hash  (d <= 16384): tasks = (row, slice of its entries) sized to ~max(64K, 8 d)
//                   probes; the workgroup builds the row's table in LDS
//                   (capacity 2d..4d slots, 8 / 32 / 128 KiB classes), then each
//                   wave takes one owned entry at a time, 64 list elements per step
//   giant (d > 16384): same tasks against an n-bit bitmap of the row (global, L2)
// Counts are integers and the value is the reference's single fp64 division,
// so the output is bit-identical to the per-entry kernel in gs_scores.hip.
#include "gs_internal.hpp"

#include <type_traits>

#include <vector>

namespace gs {

static constexpr int64_t kJacLight = 32;
static constexpr int64_t kJacGiant = 16384;
static constexpr int64_t kJacTaskMin = 65536;
static constexpr int kJacClasses = 5;  // 4 LDS table sizes + bitmap
static constexpr int kJacBitmap = 4;
static constexpr int kJacUnrollDef = 4;  // list elements per lane in flight
// the big-table classes run 1-2 workgroups per CU: more list loads in flight per lane
#ifndef GS_JAC_UNROLL_BIG
#define GS_JAC_UNROLL_BIG 8
#endif
static constexpr int kJacMaxEnt = 1024;  // entries per task (LDS staging)
static constexpr int64_t kJacSmall = 16;  // d_v <= this: 16-lane groups

__device__ __forceinline__ bool jac_owns(int64_t du, int64_t dv, int32_t u, int32_t v) {
    return du > dv || (du == dv && u <= v);
}

__device__ __forceinline__ double jac_value(int64_t inter, int64_t du, int64_t dv) {
    double uni = (double)du + (double)dv - (double)inter;
    return uni > 0.0 ? (double)inter / uni : 0.0;
}

// counts != 0: the raw |N(u) ∩ N(v)| (gs_common_neighbors) instead of the ratio
__device__ __forceinline__ double jac_out(int counts, int64_t inter, int64_t du, int64_t dv) {
    return counts ? (double)inter : jac_value(inter, du, dv);
}

// Where a pair's result goes: both CSR entries of the full score vector (out,
// rev = tpos), or -- the sharded form (gs_jaccard_part_counts) -- the raw count
// into this part's compact owner-entry array cc[opre[e] - obase]
struct JacSink {
    double *out;
    const int64_t *rev;
    int counts;
    uint32_t *cc;
    const int64_t *opre;
    int64_t obase;
    __device__ __forceinline__ void put(int64_t e, int64_t cnt, int64_t du, int64_t dv) const {
        if (cc) {
            cc[opre[e] - obase] = (uint32_t)cnt;
            return;
        }
        const double val = jac_out(counts, cnt, du, dv);
        out[e] = val;
        out[rev[e]] = val;
    }
};

__host__ __device__ __forceinline__ int jac_class(int64_t d) {
    if (d <= kJacLight) return -1;
    if (d <= 1024) return 0;
    if (d <= 4096) return 1;
    if (d <= 8192) return 2;
    if (d <= kJacGiant) return 3;
    return kJacBitmap;
}

// probes per task: enough to amortise clearing the C-slot table and the d_u inserts
__host__ __device__ __forceinline__ int64_t jac_task_probes(int k, int64_t du) {
    const int64_t tab = k == 0 ? 2048 : k == 1 ? 8192 : k == 2 ? 16384 : k == 3 ? 32768 : 0;
    int64_t t = 16 * tab > 8 * du ? 16 * tab : 8 * du;
    return t > kJacTaskMin ? t : kJacTaskMin;
}

// task count of a row of class k >= 0 with owned-entry probe work w (sum of d_v)
__host__ __device__ __forceinline__ int64_t jac_row_tasks(int k, int64_t du, int64_t w) {
    if (k < 0 || !w) return 0;
    const int64_t t = jac_task_probes(k, du);
    int64_t nt = (w + t - 1) / t;
    const int64_t ne = (du + kJacMaxEnt - 1) / kJacMaxEnt;
    if (nt < ne) nt = ne;
    if (nt > du) nt = du;
    return nt;
}

// per row of [r0, r1) (one wave each): class, task count (work = sum of d_v over
// owned entries); tot[0..4] = per-class task totals of the range, tot[5] = its rows
// with bitmap tasks.  A part of the sharded form plans only its own rows.
__global__ void __launch_bounds__(256) k_jac_plan(const int64_t *__restrict__ ip,
                                                  const int32_t *__restrict__ ix, int64_t r0,
                                                  int64_t r1, int8_t *__restrict__ cls,
                                                  int32_t *__restrict__ ntask,
                                                  unsigned long long *__restrict__ tot) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    unsigned long long mine[kJacClasses + 1] = {};  // lane 0: this wave's task totals
    for (int64_t u = r0 + w0; u < r1; u += nw) {
        const int64_t a = ip[u], du = ip[u + 1] - a;
        const int k = jac_class(du);
        int64_t w = 0;
        if (k >= 0) {
            for (int64_t e = a + lane; e < a + du; e += 64) {
                const int32_t v = ix[e];
                const int64_t dv = ip[v + 1] - ip[v];
                if (jac_owns(du, dv, (int32_t)u, v)) w += dv;
            }
            for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
        }
        if (lane == 0) {
            const int64_t nt = jac_row_tasks(k, du, w);
            cls[u] = (int8_t)k;
            ntask[u] = (int32_t)nt;
            if (nt) {
#pragma unroll
                for (int q = 0; q < kJacClasses; ++q) mine[q] += q == k ? (unsigned long long)nt : 0ull;
                mine[kJacClasses] += k == kJacBitmap ? 1ull : 0ull;
            }
        }
    }
    __shared__ unsigned long long red[kJacClasses + 1];
    if (threadIdx.x < kJacClasses + 1) red[threadIdx.x] = 0;
    __syncthreads();
    if (lane == 0)
#pragma unroll
        for (int q = 0; q <= kJacClasses; ++q)
            if (mine[q]) atomicAdd(&red[q], mine[q]);
    __syncthreads();
    if (threadIdx.x < kJacClasses + 1 && red[threadIdx.x]) atomicAdd(&tot[threadIdx.x], red[threadIdx.x]);
}

// Sharded form (gs_jaccard_shares): per-row intersection work of the owner entries
// -- light rows d_u + d_v per owned entry (the merge), other rows d_v per owned entry
// (the probes) plus d_u per task (the table build) -- for cutting the rows into
// contiguous ranges of equal work
__global__ void __launch_bounds__(256) k_jac_rowwork(const int64_t *__restrict__ ip,
                                                     const int32_t *__restrict__ ix, int64_t n,
                                                     int64_t *__restrict__ work) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t u = w0; u < n; u += nw) {
        const int64_t a = ip[u], du = ip[u + 1] - a;
        const int k = jac_class(du);
        int64_t w = 0;
        for (int64_t e = a + lane; e < a + du; e += 64) {
            const int32_t v = ix[e];
            const int64_t dv = ip[v + 1] - ip[v];
            if (jac_owns(du, dv, (int32_t)u, v)) w += k < 0 ? du + dv : dv;
        }
        for (int o = 32; o > 0; o >>= 1) w += __shfl_xor(w, o);
        if (lane == 0) work[u] = w + jac_row_tasks(k, du, w) * du;
    }
}

// owner flag of every CSR entry (1: the entry (u, v) is its pair's owner entry)
__global__ void k_jac_owner_flags(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                  const int32_t *__restrict__ rows, int64_t nnz,
                                  int64_t *__restrict__ flag) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = rows[e], v = ix[e];
        flag[e] = jac_owns(ip[u + 1] - ip[u], ip[v + 1] - ip[v], u, v) ? 1 : 0;
    }
}

// owner list (sharded form): for owner entry i (CSR order) its CSR position, its
// reverse entry and d_u + d_v, so the scatter streams them instead of reading
// both endpoints' indptr at random
__global__ void k_jac_owner_list(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                 const int32_t *__restrict__ rows, const int64_t *__restrict__ rev,
                                 const int64_t *__restrict__ opre, int64_t nnz,
                                 int32_t *__restrict__ opos, int32_t *__restrict__ orev,
                                 int32_t *__restrict__ osum) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = opre[e];
        if (opre[e + 1] == i) continue;  // not an owner entry
        const int32_t u = rows[e], v = ix[e];
        opos[i] = (int32_t)e;
        orev[i] = (int32_t)rev[e];
        osum[i] = (int32_t)((ip[u + 1] - ip[u]) + (ip[v + 1] - ip[v]));
    }
}

// cut rows: R[r] = first row u with S[u] >= total * r / P (S: exclusive prefix of the
// row work, S[n] = total), R[0] = 0, R[P] = n; then E[r] = ip[R[r]] and
// O[r] = opre[E[r]].  One thread per cut (P + 1 of them, any P: the grid covers
// them all).  out = [R | E | O], 3 (P + 1) values.
__global__ void k_jac_cuts(const int64_t *__restrict__ S, const int64_t *__restrict__ ip,
                           const int64_t *__restrict__ opre, int64_t n, int P,
                           int64_t *__restrict__ out) {
    const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r > P) return;
    const int64_t total = S[n];
    int64_t R;
    if (r == 0) R = 0;
    else if (r == P) R = n;
    else {
        const int64_t t = total * r / P;
        int64_t lo = 0, hi = n;  // first u in [0, n] with S[u] >= t
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (S[mid] >= t) hi = mid;
            else lo = mid + 1;
        }
        R = lo;
    }
    out[r] = R;
    out[P + 1 + r] = ip[R];
    out[2 * (P + 1) + r] = opre[ip[R]];
}

// sharded form: every part's counts -> both CSR entries of each pair, one thread per
// owner pair i; O[0..P] = cuts[2 (P + 1) ..].  fl(d_u + d_v) == d_u + d_v exactly, so
// the value is jac_value's bit for bit.
__global__ void k_jac_scatter_owners(const int32_t *__restrict__ opos, const int32_t *__restrict__ orev,
                                     const int32_t *__restrict__ osum, const int64_t *__restrict__ cuts,
                                     int P, const uint32_t *__restrict__ cc, int64_t stride,
                                     int64_t nown, double *__restrict__ out) {
    const int64_t *O = cuts + 2 * (P + 1);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nown;
         i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = P - 1;  // last part r with O[r] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (O[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const int64_t cnt = cc[lo * stride + (i - O[lo])];
        const double uni = (double)osum[i] - (double)cnt;
        const double val = uni > 0.0 ? (double)cnt / uni : 0.0;
        out[opos[i]] = val;
        out[orev[i]] = val;
    }
}

// sharded form, graphs past int32 positions: every part's counts -> both CSR entries
__global__ void k_jac_from_counts(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                  const int32_t *__restrict__ rows, const int64_t *__restrict__ rev,
                                  const int64_t *__restrict__ opre, const int64_t *__restrict__ cuts,
                                  int P, const uint32_t *__restrict__ cc, int64_t stride,
                                  int64_t nnz, double *__restrict__ out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = rows[e], v = ix[e];
        const int64_t du = ip[u + 1] - ip[u], dv = ip[v + 1] - ip[v];
        if (!jac_owns(du, dv, u, v)) continue;
        int r = 0;  // part whose row range holds u: cuts[0..P] = R
        while (r + 1 < P && u >= cuts[r + 1]) ++r;
        const int64_t cnt = cc[r * stride + (opre[e] - cuts[2 * (P + 1) + r])];
        const double val = jac_value(cnt, du, dv);
        out[e] = val;
        out[rev[e]] = val;
    }
}

// rows [r0, r1): cnt / gflag indexed u - r0
__global__ void k_jac_mask(const int8_t *__restrict__ cls, const int32_t *__restrict__ ntask,
                           int64_t r0, int64_t r1, int k, int64_t *__restrict__ cnt,
                           int64_t *__restrict__ gflag) {
    for (int64_t u = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < r1;
         u += (int64_t)gridDim.x * blockDim.x) {
        const bool in = cls[u] == k;
        cnt[u - r0] = in ? ntask[u] : 0;
        if (gflag) gflag[u - r0] = (in && ntask[u] > 0) ? 1 : 0;
    }
}

// tasks of class k in row order; giant rows also get their bitmap slot
__global__ void k_jac_emit(const int8_t *__restrict__ cls, const int32_t *__restrict__ ntask,
                           const int64_t *__restrict__ off, const int64_t *__restrict__ goff,
                           int64_t r0, int64_t r1, int k, int32_t *__restrict__ trow,
                           int32_t *__restrict__ ti, int32_t *__restrict__ tslot,
                           int32_t *__restrict__ grow) {
    for (int64_t u = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < r1;
         u += (int64_t)gridDim.x * blockDim.x) {
        if (cls[u] != k) continue;
        const int32_t nt = ntask[u];
        if (!nt) continue;
        const int64_t o = off[u - r0];
        const int32_t g = goff ? (int32_t)goff[u - r0] : 0;
        if (goff) grow[g] = (int32_t)u;
        for (int32_t i = 0; i < nt; ++i) {
            trow[o + i] = (int32_t)u;
            ti[o + i] = i;
            if (tslot) tslot[o + i] = g;
        }
    }
}

// light rows: one thread per owned entry, merge of two <= 32-long sorted lists
__global__ void __launch_bounds__(256) k_jac_light(const int64_t *__restrict__ ip,
                                                   const int32_t *__restrict__ ix,
                                                   const int32_t *__restrict__ rows,
                                                   int64_t e0, int64_t e1, JacSink sk) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = rows[e];
        const int64_t a = ip[u], du = ip[u + 1] - a;
        if (du > kJacLight) continue;
        const int32_t v = ix[e];
        const int64_t b = ip[v], dv = ip[v + 1] - b;
        if (!jac_owns(du, dv, u, v)) continue;
        int64_t i = 0, j = 0, cnt = 0;
        while (i < du && j < dv) {
            const int32_t x = ix[a + i], y = ix[b + j];
            cnt += (x == y);
            i += (x <= y);
            j += (y <= x);
        }
        sk.put(e, cnt, du, dv);
    }
}

// GS_JAC_FASTHASH (default 1): the tables' multiplicative hash with a 24-bit odd multiplier
// (v_mul_u32_u24, full rate, instead of v_mul_lo_u32, quarter rate): (x * K) mod 2^b is
// still a bijection of [0, 2^b) for the quotient tables, whose ids are < 2^24
// (jac_qparams); the int32 tables compare whole ids, so any hash is exact there
#ifndef GS_JAC_FASTHASH
#define GS_JAC_FASTHASH 1
#endif
static constexpr uint32_t kJacMul24 = 0x9E3779u;  // odd
__device__ __forceinline__ uint32_t jac_mul(uint32_t x) {
#if GS_JAC_FASTHASH
    return __umul24(x, kJacMul24);
#else
    return x * 2654435761u;
#endif
}
__device__ __forceinline__ uint32_t jac_hash(int32_t x) { return jac_mul((uint32_t)x); }

// Owned entries of a task, staged in LDS: (list base, length, entry offset).
// Entries with d_v > kJacSmall fill the front and are taken one per wave;
// short ones fill the back and are taken four per wave (16-lane groups).
struct JacStage {
    int64_t b[kJacMaxEnt];
    int32_t dv[kJacMaxEnt];
    int16_t off[kJacMaxEnt];
    int nbig, nsmall;
};

__device__ __forceinline__ void jac_stage(const int64_t *__restrict__ ip,
                                          const int32_t *__restrict__ ix, int32_t u, int64_t du,
                                          int64_t lo, int64_t hi, JacStage &st) {
    for (int64_t e = lo + threadIdx.x; e < hi; e += blockDim.x) {
        const int32_t v = ix[e];
        const int64_t b = ip[v], dv = ip[v + 1] - b;
        if (!jac_owns(du, dv, u, v)) continue;
        const int k = dv > kJacSmall ? atomicAdd(&st.nbig, 1)
                                     : kJacMaxEnt - 1 - atomicAdd(&st.nsmall, 1);
        st.b[k] = b;
        st.dv[k] = (int32_t)dv;
        st.off[k] = (int16_t)(e - lo);
    }
}

// Membership tests in two steps, so a lane can have every first read in
// flight before it resolves any: first(x) issues the read, done(x, s)
// finishes (following full buckets of the LDS table when it must).
struct JacHashProbe {
    const int4 *tab;
    uint32_t shift, mask;
    struct S {
        int4 q;
        uint32_t h;
    };
    __device__ __forceinline__ S first(int32_t x) const {
        const uint32_t h = jac_hash(x) >> shift;
        return S{tab[h], h};
    }
    __device__ __forceinline__ bool done(int32_t x, S s) const {
        while (true) {
            if (s.q.x == x || s.q.y == x || s.q.z == x || s.q.w == x) return true;
            if (s.q.w == -1) return false;
            s.h = (s.h + 1) & mask;
            s.q = tab[s.h];
        }
    }
    // the home bucket alone, branch-free: hit, or more = the search must go on (done())
    __device__ __forceinline__ bool check1(int32_t x, S s, bool &more) const {
        const bool hit = s.q.x == x || s.q.y == x || s.q.z == x || s.q.w == x;
        more = !hit && s.q.w != -1;
        return hit;
    }
};

struct JacBitProbe {
    const uint32_t *m;
    struct S {
        uint32_t w;
    };
    __device__ __forceinline__ S first(int32_t x) const { return S{m[x >> 5]}; }
    __device__ __forceinline__ bool done(int32_t x, S s) const { return (s.w >> (x & 31)) & 1u; }
    __device__ __forceinline__ bool check1(int32_t x, S s, bool &more) const {
        more = false;
        return done(x, s);
    }
};

// Probe phase shared by the LDS-table and bitmap kernels (after jac_stage and
// a barrier).  The d_u of the owner and each entry's d_v give the union.
// UL list elements per lane are loaded at once (the global reads are what the
// loop waits on), then probed UP at a time (the probe state is what costs
// registers).  Measured and dropped (profiles/r04g_*, r04t_*, r04u_*): skipping
// the all-masked 64-element steps; a software-pipelined loop with the next step's
// loads in flight during this step's probes; and cutting long lists into chunks
// the waves take in turn (the slowest wave of a 16K / 32K task had ~1.45x the mean
// steps) -- the last two are 6-14 % faster per class run alone and 2-6 % slower
// with the classes overlapping on their streams, which fill each other's idle
// waves already.
#ifndef GS_JAC_MASKLOAD
#define GS_JAC_MASKLOAD 1
#endif
#ifndef GS_JAC_FASTPROBE
#define GS_JAC_FASTPROBE 1
#endif
template <class Probe, int UL = kJacUnrollDef, int UP = UL>
__device__ __forceinline__ void jac_probe_staged(const int32_t *__restrict__ ix, int64_t du,
                                                 int64_t lo, const JacStage &st,
                                                 const JacSink &sk, const Probe &pr) {
    static_assert(UL % UP == 0, "probe groups split the loaded elements");
    static_assert(64 * UL <= kIxPad, "unconditional list steps stay inside the index padding");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    using gi32 = __attribute__((address_space(1))) const int32_t;  // global, not flat
    // one step: U list elements per lane loaded (all in flight before the first probe),
    // lanes past d_v masked (MASK), then probed in groups of min(UP, U)
    auto step = [&](auto Uc, auto MASKc, gi32 *lp, int32_t left, int64_t &cnt) {
        constexpr int U = decltype(Uc)::value;
        constexpr bool MASK = decltype(MASKc)::value;
        constexpr int P = UP < U ? UP : U;
        int32_t xs[U];
#pragma unroll
        for (int t = 0; t < U; ++t) {
            if constexpr (MASK && GS_JAC_MASKLOAD) {  // lanes past d_v issue no load (exec-masked)
                xs[t] = -1;
                if (lane + t * 64 < left) xs[t] = lp[t * 64];
            } else if constexpr (MASK) {  // (round 5: every lane loads, then the mask)
                const int32_t x = lp[t * 64];
                xs[t] = lane + t * 64 < left ? x : -1;
            } else {
                xs[t] = lp[t * 64];
            }
        }
#pragma unroll
        for (int g = 0; g < U; g += P) {
            typename Probe::S ps[P];
#pragma unroll
            for (int t = 0; t < P; ++t) ps[t] = pr.first(xs[g + t] >= 0 ? xs[g + t] : 0);
            if constexpr (GS_JAC_FASTPROBE) {
                // the home buckets branch-free; the rare lanes whose search goes on take
                // done() under one wave-uniform branch (a per-element search loop costs
                // ~20 scalar mask operations per element even when it ends at once)
                bool hit[P], more[P], any = false;
#pragma unroll
                for (int t = 0; t < P; ++t) {
                    hit[t] = pr.check1(xs[g + t], ps[t], more[t]);
                    more[t] = more[t] && xs[g + t] >= 0;
                    any = any || more[t];
                }
                if (__builtin_amdgcn_ballot_w64(any)) {
#pragma unroll
                    for (int t = 0; t < P; ++t)
                        if (more[t]) hit[t] = pr.done(xs[g + t], ps[t]);
                }
#pragma unroll
                for (int t = 0; t < P; ++t) cnt += __popcll(__ballot(xs[g + t] >= 0 && hit[t]));
            } else {
#pragma unroll
            for (int t = 0; t < P; ++t) {
                const bool hit = xs[g + t] >= 0 && pr.done(xs[g + t], ps[t]);
                cnt += __popcll(__ballot(hit));
            }
            }
        }
    };
    using T1 = std::true_type;
    using F0 = std::false_type;
    for (int k = wave; k < st.nbig; k += nw) {
        const int32_t dv = __builtin_amdgcn_readfirstlane(st.dv[k]);
        // the list's base is wave-uniform: loads from a scalar base, one lane offset and
        // immediate step offsets.  Whole 64 UL-element steps first (no mask), then one
        // step of the fewest loads (1, 2, 4 .. UL per lane) that covers the rest, its
        // lanes past d_v masked -- they read at most 63 entries past the list (the next
        // rows', or the kIxPad padding after the last row).  (Round 4 read every list in
        // 64 UL-element steps: up to 511 entries past a short list, 98 GB fetched per
        // R-MAT-22 call against ~50 GB probed.)
        const uint64_t lb = (uint64_t)(ix + st.b[k]);
        gi32 *lst = (gi32 *)(
            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lb) |
            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lb >> 32)) << 32);
        int64_t cnt = 0;
        int32_t j0 = 0;
        for (; j0 + 64 * UL <= dv; j0 += 64 * UL)
            step(std::integral_constant<int, UL>{}, F0{}, lst + (uint32_t)(j0 + lane), 64 * UL, cnt);
        const int32_t rem = dv - j0;  // wave-uniform
        gi32 *lp = lst + (uint32_t)(j0 + lane);
        if (rem > 0) {
            if (rem <= 64) step(std::integral_constant<int, 1>{}, T1{}, lp, rem, cnt);
            else if (UL >= 2 && rem <= 128) step(std::integral_constant<int, (UL >= 2 ? 2 : 1)>{}, T1{}, lp, rem, cnt);
            else if (UL >= 4 && rem <= 256) step(std::integral_constant<int, (UL >= 4 ? 4 : 1)>{}, T1{}, lp, rem, cnt);
            else step(std::integral_constant<int, UL>{}, T1{}, lp, rem, cnt);
        }
        if (lane == 0) sk.put(lo + st.off[k], cnt, du, dv);
    }
    const int grp = lane >> 4, gl = lane & 15;
    const uint64_t gmask = 0xFFFFull << (16 * grp);
    for (int r = wave * 4; r < st.nsmall; r += nw * 4) {
        const int idx = r + grp;
        const bool ok = idx < st.nsmall;
        const int k = kJacMaxEnt - 1 - (ok ? idx : 0);
        const int64_t dv = ok ? st.dv[k] : 0;
        const int32_t x = gl < dv ? ix[st.b[k] + gl] : -1;
        const typename Probe::S ps = pr.first(x >= 0 ? x : 0);
        bool hit;
        if constexpr (GS_JAC_FASTPROBE) {
            bool more;
            hit = pr.check1(x, ps, more);
            more = more && x >= 0;
            if (__builtin_amdgcn_ballot_w64(more))
                if (more) hit = pr.done(x, ps);
            hit = hit && x >= 0;
        } else {
            hit = x >= 0 && pr.done(x, ps);
        }
        const int64_t cnt = __popcll(__ballot(hit) & gmask);
        if (ok && gl == 0) sk.put(lo + st.off[k], cnt, du, dv);
    }
}

__device__ __forceinline__ void jac_task_range(const int64_t *__restrict__ ip,
                                               const int32_t *__restrict__ ntask, int32_t u,
                                               int32_t i, int64_t &a, int64_t &du, int64_t &lo,
                                               int64_t &hi) {
    a = ip[u];
    du = ip[u + 1] - a;
    const int64_t nt = ntask[u];
    lo = a + du * i / nt;
    hi = a + du * (i + 1) / nt;
}

// one task per workgroup; table of C int32 slots in LDS (empty = -1)
template <int C>
__global__ void __launch_bounds__(1024) k_jac_hash(const int64_t *__restrict__ ip,
                                                   const int32_t *__restrict__ ix,
                                                   const int32_t *__restrict__ ntask,
                                                   const int32_t *__restrict__ trow,
                                                   const int32_t *__restrict__ ti, int64_t t0,
                                                   JacSink sk) {
    // 4-slot buckets (one 16-B LDS read per probe step); a bucket fills from
    // slot 0 up, so a bucket with a free slot 3 ends an unsuccessful search
    __shared__ int4 tab[C / 4];
    __shared__ JacStage st;
    const int64_t t = t0 + blockIdx.x;
    const int32_t u = trow[t];
    int64_t a, du, lo, hi;
    jac_task_range(ip, ntask, u, ti[t], a, du, lo, hi);
    if (threadIdx.x == 0) st.nbig = st.nsmall = 0;
    for (int s = threadIdx.x; s < C / 4; s += blockDim.x) tab[s] = make_int4(-1, -1, -1, -1);
    __syncthreads();
    jac_stage(ip, ix, u, du, lo, hi, st);
    constexpr uint32_t shift = 32 - __builtin_ctz(C / 4);
    constexpr uint32_t mask = C / 4 - 1;
    int32_t *slots = reinterpret_cast<int32_t *>(tab);
    for (int64_t e = a + threadIdx.x; e < a + du; e += blockDim.x) {
        const int32_t x = ix[e];
        uint32_t h = jac_hash(x) >> shift;
        bool done = false;
        while (!done) {
#pragma unroll
            for (int q = 0; q < 4 && !done; ++q) {
                const int32_t prev = atomicCAS(&slots[h * 4 + q], -1, x);
                done = prev == -1 || prev == x;
            }
            h = (h + 1) & mask;
        }
    }
    __syncthreads();
    constexpr int U = C >= 16384 ? GS_JAC_UNROLL_BIG : kJacUnrollDef;
    jac_probe_staged<JacHashProbe, U>(ix, du, lo, st, sk, JacHashProbe{tab, shift, mask});
}

// Quotient tables (classes in GS_JAC_Q16, when the ids fit): 16-bit slots, so the
// same LDS holds twice the slots -- half the load factor, and the 32K-slot class
// runs two workgroups per CU instead of one.  h = (x * K) mod 2^b (jac_mul) is a
// bijection of [0, 2^b) (odd multiplier, n <= 2^b); its top bits pick the home
// bucket, the low qb bits (the remainder) go into the slot with the bucket's
// distance from home: slot = (d + 1) << qb | rem, 0 = empty.  (bucket, slot)
// gives h back, so a match is exact.  Buckets of 8 slots (one 16-B LDS read per
// probe step) fill from slot 0 up; a free slot 7 ends an unsuccessful search.
// An insert that would go past the largest distance a slot can encode flags the
// task, which then probes the owner's sorted list instead (never seen in practice).
#ifndef GS_JAC_Q16
#define GS_JAC_Q16 0xE  // classes 1, 2, 3
#endif
#ifndef GS_JAC_UNROLL_Q8  // the two-workgroups-per-CU 32K class: 64 VGPRs
#define GS_JAC_UNROLL_Q8 4
#endif
#ifndef GS_JAC_LOADS_Q8  // ... with this many list loads per lane in flight
#define GS_JAC_LOADS_Q8 8
#endif

// any zero 16-bit half in v
__device__ __forceinline__ uint32_t jac_hz16(uint32_t v) {
    return (v - 0x00010001u) & ~v & 0x80008000u;
}

// any of the 8 16-bit slots of a bucket equal to t (t2 = t in both halves).  GS_JAC_PKMIN
// (default 1): the packed 16-bit minimum of the four XORed words (v_pk_min_u16) has a zero
// half iff some slot matches -- 4 XOR + 3 packed minima + one zero-half test instead of
// four zero-half tests and their ORs
#ifndef GS_JAC_PKMIN
#define GS_JAC_PKMIN 1
#endif
__device__ __forceinline__ bool jac_bucket_has(const uint4 &q, uint32_t t2) {
#if GS_JAC_PKMIN
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 a = __builtin_bit_cast(u16x2, q.x ^ t2), b = __builtin_bit_cast(u16x2, q.y ^ t2);
    const u16x2 c = __builtin_bit_cast(u16x2, q.z ^ t2), d = __builtin_bit_cast(u16x2, q.w ^ t2);
    const u16x2 m = __builtin_elementwise_min(__builtin_elementwise_min(a, b), __builtin_elementwise_min(c, d));
    return jac_hz16(__builtin_bit_cast(uint32_t, m)) != 0;
#else
    return (jac_hz16(q.x ^ t2) | jac_hz16(q.y ^ t2) | jac_hz16(q.z ^ t2) | jac_hz16(q.w ^ t2)) != 0;
#endif
}

struct JacQParams {
    uint32_t hmask, qb, rmask, dmax;  // 2^b - 1, remainder bits, 2^qb - 1, largest distance
};

struct JacQProbe {
    const uint4 *tab;
    JacQParams p;
    uint32_t nbm;  // buckets - 1
    struct S {
        uint4 q;
        uint32_t h;
    };
    __device__ __forceinline__ S first(int32_t x) const {
        const uint32_t h = jac_mul((uint32_t)x) & p.hmask;
        return S{tab[h >> p.qb], h};
    }
    __device__ __forceinline__ bool done(int32_t, S s) const {
        const uint32_t home = s.h >> p.qb, rem = s.h & p.rmask;
        for (uint32_t d = 0;;) {
            const uint32_t t = ((d + 1) << p.qb) | rem, t2 = t | (t << 16);
            if (jac_bucket_has(s.q, t2)) return true;
            if ((s.q.w >> 16) == 0 || ++d > p.dmax) return false;
            s.q = tab[(home + d) & nbm];
        }
    }
    __device__ __forceinline__ bool check1(int32_t, S s, bool &more) const {
        const uint32_t t = (1u << p.qb) | (s.h & p.rmask), t2 = t | (t << 16);
        const bool hit = jac_bucket_has(s.q, t2);
        more = !hit && (s.q.w >> 16) != 0 && p.dmax >= 1;
        return hit;
    }
};

// the overflow path: binary search of the owner's sorted neighbour list
struct JacSortedProbe {
    const int32_t *row;
    int64_t du;
    struct S {};
    __device__ __forceinline__ S first(int32_t) const { return S{}; }
    __device__ __forceinline__ bool check1(int32_t, S, bool &more) const {
        more = true;
        return false;
    }
    __device__ __forceinline__ bool done(int32_t x, S) const {
        int64_t lo = 0, hi = du;
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (row[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        return lo < du && row[lo] == x;
    }
};

// one task per workgroup; C 16-bit slots in LDS; MINW waves per SIMD
template <int C, int NT, int MINW>
__global__ void __launch_bounds__(NT, MINW) k_jac_hashq(const int64_t *__restrict__ ip,
                                                        const int32_t *__restrict__ ix,
                                                        const int32_t *__restrict__ ntask,
                                                        const int32_t *__restrict__ trow,
                                                        const int32_t *__restrict__ ti, int64_t t0,
                                                        JacQParams qp, JacSink sk) {
    constexpr int NB = C / 8;
    __shared__ uint4 tab[NB];
    __shared__ JacStage st;
    __shared__ int ovf;
    const int64_t t = t0 + blockIdx.x;
    const int32_t u = trow[t];
    int64_t a, du, lo, hi;
    jac_task_range(ip, ntask, u, ti[t], a, du, lo, hi);
    if (threadIdx.x == 0) st.nbig = st.nsmall = ovf = 0;
    for (int s = threadIdx.x; s < NB; s += blockDim.x) tab[s] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    jac_stage(ip, ix, u, du, lo, hi, st);
    uint32_t *words = reinterpret_cast<uint32_t *>(tab);
    for (int64_t e = a + threadIdx.x; e < a + du; e += blockDim.x) {
        const uint32_t h = jac_mul((uint32_t)ix[e]) & qp.hmask;
        const uint32_t home = h >> qp.qb, rem = h & qp.rmask;
        bool in = false;
        for (uint32_t d = 0; d <= qp.dmax && !in; ++d) {
            const uint32_t ent = ((d + 1) << qp.qb) | rem;
            uint32_t *w = words + ((home + d) & (NB - 1)) * 4;
            for (int q = 0; q < 8 && !in; ++q) {
                const int sh = (q & 1) * 16;
                uint32_t cur = 0;  // guess: the word is empty
                while (true) {
                    if ((cur >> sh) & 0xFFFFu) break;  // slot taken: the next one
                    const uint32_t prev = atomicCAS(&w[q >> 1], cur, cur | (ent << sh));
                    if (prev == cur) {
                        in = true;
                        break;
                    }
                    cur = prev;
                }
            }
        }
        if (!in) ovf = 1;
    }
    __syncthreads();
    if (ovf)
        jac_probe_staged<JacSortedProbe, 1>(ix, du, lo, st, sk, JacSortedProbe{ix + a, du});
    else
        jac_probe_staged<JacQProbe, (MINW >= 8 ? GS_JAC_LOADS_Q8 : GS_JAC_UNROLL_BIG),
                         (MINW >= 8 ? GS_JAC_UNROLL_Q8 : GS_JAC_UNROLL_BIG)>(ix, du, lo, st, sk,
                                                                             JacQProbe{tab, qp, NB - 1});
}

// quotient-table parameters for C 16-bit slots and ids < n; false when the
// remainder leaves too few distance bits (n past ~2^24)
static bool jac_qparams(int64_t n, int C, JacQParams &p) {
    int b = 1;
    while (b < 31 && ((int64_t)1 << b) < n) ++b;
    const int bb = __builtin_ctz((unsigned)(C / 8));
    if (b < bb) b = bb;
    const int qb = b - bb;
    if (16 - qb < 4) return false;
    p.hmask = b >= 32 ? 0xFFFFFFFFu : (uint32_t)(((uint64_t)1 << b) - 1);
    p.qb = (uint32_t)qb;
    p.rmask = (1u << qb) - 1;
    uint32_t dmax = (1u << (16 - qb)) - 2;
    if (dmax > (uint32_t)(C / 8 - 1)) dmax = (uint32_t)(C / 8 - 1);
    p.dmax = dmax;
    return true;
}

__global__ void k_jac_bitmap_build(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                                   const int32_t *__restrict__ grow, int32_t g0, int64_t words,
                                   uint32_t *__restrict__ bm) {
    const int32_t u = grow[g0 + blockIdx.y];
    uint32_t *m = bm + (int64_t)blockIdx.y * words;
    for (int64_t e = ip[u] + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ip[u + 1];
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t x = ix[e];
        atomicOr(&m[x >> 5], 1u << (x & 31));
    }
}

__global__ void __launch_bounds__(1024) k_jac_bitmap(const int64_t *__restrict__ ip,
                                                     const int32_t *__restrict__ ix,
                                                     const int32_t *__restrict__ ntask,
                                                     const int32_t *__restrict__ trow,
                                                     const int32_t *__restrict__ ti,
                                                     const int32_t *__restrict__ tslot,
                                                     int64_t t0, int32_t g0, int64_t words,
                                                     const uint32_t *__restrict__ bm, JacSink sk) {
    const int64_t t = t0 + blockIdx.x;
    const int32_t u = trow[t];
    int64_t a, du, lo, hi;
    jac_task_range(ip, ntask, u, ti[t], a, du, lo, hi);
    const uint32_t *m = bm + (int64_t)(tslot[t] - g0) * words;
    __shared__ JacStage st;
    if (threadIdx.x == 0) st.nbig = st.nsmall = 0;
    __syncthreads();
    jac_stage(ip, ix, u, du, lo, hi, st);
    __syncthreads();
    jac_probe_staged(ix, du, lo, st, sk, JacBitProbe{m});
}

// B_J for a symmetric graph: 8 * sum_u d_u^2 + 12 * nnz
__global__ void k_jac_bytes(const int64_t *__restrict__ ip, int64_t n,
                            unsigned long long *__restrict__ acc) {
    unsigned long long s = 0;
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long d = (unsigned long long)(ip[u + 1] - ip[u]);
        s += d * d;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(acc, s);
}

// Row ranges of the sharded form (cached per graph and part count): R[0..P] cut
// rows, E[r] = ip[R[r]], O[r] = owner entries before E[r]; opre (device) = the
// exclusive prefix of the owner flags over the CSR entries
const JacShares &jaccard_shares(gs_ctx *c, int P) {
    Graph &g = c->g;
    if (c->jac_epoch != g.epoch) {
        c->jac_shares.clear();
        c->jac_epoch = g.epoch;
    }
    auto it = c->jac_shares.find(P);
    if (it != c->jac_shares.end()) return it->second;
    const int64_t n = g.n, nnz = g.nnz;
    hipStream_t st = c->stream;
    const int64_t *ip = g.indptr.as<int64_t>();
    const int32_t *ix = g.indices.as<int32_t>();
    auto *opre = (int64_t *)c->buf("jac_opre").ensure(sizeof(int64_t) * (nnz + 1));
    if (c->jac_shares.empty()) {  // the owner prefix is the same for every P
        auto *fl = (int64_t *)c->buf("jac_oflag").ensure(sizeof(int64_t) * (nnz + 1));
        GS_HIP(hipMemsetAsync(fl + nnz, 0, sizeof(int64_t), st));
        if (nnz)
            k_jac_owner_flags<<<grid_for(nnz, 256, 65536), 256, 0, st>>>(ip, ix, g.rows.as<int32_t>(),
                                                                         nnz, fl);
        exclusive_scan_i64(c, fl, opre, nnz + 1);
        c->buf("jac_oflag").release();
        if (nnz < (int64_t)INT32_MAX) {
            int64_t nown = 0;
            GS_HIP(hipMemcpyAsync(&nown, opre + nnz, sizeof(int64_t), hipMemcpyDeviceToHost, st));
            GS_HIP(hipStreamSynchronize(st));
            const size_t b = sizeof(int32_t) * (size_t)(nown ? nown : 1);
            auto *opos = (int32_t *)c->buf("jac_opos").ensure(b);
            auto *orev = (int32_t *)c->buf("jac_orev").ensure(b);
            auto *osum = (int32_t *)c->buf("jac_osum").ensure(b);
            if (nnz)
                k_jac_owner_list<<<grid_for(nnz, 256, 65536), 256, 0, st>>>(
                    ip, ix, g.rows.as<int32_t>(), g.tpos.as<int64_t>(), opre, nnz, opos, orev, osum);
            GS_HIP(hipGetLastError());
        }
    }
    auto *work = (int64_t *)c->buf("jac_work").ensure(sizeof(int64_t) * (n + 1));
    auto *S = (int64_t *)c->buf("jac_wpre").ensure(sizeof(int64_t) * (n + 1));
    GS_HIP(hipMemsetAsync(work + n, 0, sizeof(int64_t), st));
    if (n) k_jac_rowwork<<<grid_for(n, 4, 4096), 256, 0, st>>>(ip, ix, n, work);
    exclusive_scan_i64(c, work, S, n + 1);
    auto *dcut = (int64_t *)c->buf("jac_cutbuf").ensure(sizeof(int64_t) * 3 * (P + 1));
    k_jac_cuts<<<(unsigned)((P + 1 + 127) / 128), 128, 0, st>>>(S, ip, opre, n, P, dcut);
    GS_HIP(hipGetLastError());
    JacShares sh;
    sh.cuts.resize(3 * (P + 1));
    GS_HIP(hipMemcpyAsync(sh.cuts.data(), dcut, sizeof(int64_t) * 3 * (P + 1), hipMemcpyDeviceToHost, st));
    GS_HIP(hipStreamSynchronize(st));
    c->buf("jac_work").release();
    c->buf("jac_wpre").release();
    return c->jac_shares.emplace(P, std::move(sh)).first->second;
}

// Whole-graph Jaccard of a symmetric graph into device out[nnz], or part
// `part` of `nparts` of it: the owner entries of that part's rows (jaccard_shares),
// both CSR entries of each pair written into out (every other entry 0.0, so the
// nparts outputs sum to the whole) -- or, with cc, the raw counts into the part's
// compact owner-entry array (gs_jaccard_part_counts).
void jaccard_symmetric(gs_ctx *c, double *out, int part, int nparts, int counts, uint32_t *cc) {
    Graph &g = c->g;
    const int64_t n = g.n, nnz = g.nnz;
    if (!nnz) return;
    hipStream_t st = c->stream;
    const int64_t *ip = g.indptr.as<int64_t>();
    const int32_t *ix = g.indices.as<int32_t>();
    const int64_t *rev = g.tpos.as<int64_t>();
    int64_t r0 = 0, r1 = n, e0 = 0, e1 = nnz, obase = 0;
    if (nparts > 1) {
        const JacShares &sh = jaccard_shares(c, nparts);
        r0 = sh.R(part), r1 = sh.R(part + 1);
        e0 = sh.E(part), e1 = sh.E(part + 1);
        obase = sh.O(part);
    }
    if (nparts > 1 && !cc) GS_HIP(hipMemsetAsync(out, 0, sizeof(double) * nnz, st));
    JacSink sk{out, rev, counts, cc, cc ? c->buf("jac_opre").as<int64_t>() : nullptr, obase};
    double algo = 0.0;
    if (c->profiling) {
        if (c->jac_bytes_epoch != g.epoch) {  // sum of degrees^2, once per graph
            auto *acc = (unsigned long long *)c->buf("jac_bytes").ensure(8);
            GS_HIP(hipMemsetAsync(acc, 0, 8, st));
            k_jac_bytes<<<grid_for(n, 256, 4096), 256, 0, st>>>(ip, n, acc);
            unsigned long long s = 0;
            GS_HIP(hipMemcpyAsync(&s, acc, 8, hipMemcpyDeviceToHost, st));
            GS_HIP(hipStreamSynchronize(st));
            c->jac_bytes_sum = (double)s;
            c->jac_bytes_epoch = g.epoch;
        }
        algo = (8.0 * c->jac_bytes_sum + 12.0 * (double)nnz) * (nnz ? (double)(e1 - e0) / (double)nnz : 0.0);
    }
    // the hash classes run concurrently on side streams (a class of big LDS tables
    // fills one or two workgroups per CU; the others use the rest): each gets its own
    // task lists; the bitmap class stays on the context stream
    bool conc = true;
    if (const char *e = getenv("GSPARSE_JAC_CONCURRENT")) conc = atoi(e) != 0;
    // The plan (row classes, per-class task lists, bitmap batches) is a function of the
    // graph and the part's rows only: a repeated call on the same rows launches the class
    // kernels from the kept task lists -- no planning kernels, no host round trip.  (With
    // the classes sharing one task-list buffer, GSPARSE_JAC_CONCURRENT=0, every call plans.)
    const std::vector<int64_t> pkey = {g.epoch, r0, r1, n, nnz};
    const bool cached = conc && c->jac_plan_key == pkey;
    if (!cached) c->jac_plan_key.clear();
    hipEvent_t t0 = prof_begin(c);
    auto *cls = (int8_t *)c->buf("jac_cls").ensure(n);
    auto *ntask = (int32_t *)c->buf("jac_ntask").ensure(sizeof(int32_t) * n);
    auto *cnt = (int64_t *)c->buf("jac_cnt").ensure(sizeof(int64_t) * (n + 1));
    auto *off = (int64_t *)c->buf("jac_off").ensure(sizeof(int64_t) * (n + 1));
    auto *gfl = (int64_t *)c->buf("jac_gflag").ensure(sizeof(int64_t) * (n + 1));
    auto *goff = (int64_t *)c->buf("jac_goff").ensure(sizeof(int64_t) * (n + 1));
    constexpr int kTot = kJacClasses + 1;
    auto *dtot = (unsigned long long *)c->buf("jac_tot").ensure(8 * kTot);
    const int64_t nr = r1 - r0;  // this part's rows: planned, task lists emitted
    if (!cached) {
        GS_HIP(hipMemsetAsync(dtot, 0, 8 * kTot, st));
        if (nr) k_jac_plan<<<grid_for(nr, 4, 4096), 256, 0, st>>>(ip, ix, r0, r1, cls, ntask, dtot);
    }
    if (e1 > e0)
        k_jac_light<<<grid_for(e1 - e0, 256, 65536), 256, 0, st>>>(ip, ix, g.rows.as<int32_t>(), e0,
                                                                   e1, sk);
    GS_HIP(hipGetLastError());
    unsigned long long *htot = c->jac_plan_tot;
    if (!cached) {
        GS_HIP(hipMemcpyAsync(htot, dtot, 8 * kTot, hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));  // the only sync unless bitmap rows exist
        c->jac_plan_bm.clear();
    }
    int64_t tmax = 1;
    for (int k = 0; k < kJacClasses; ++k) tmax = (int64_t)htot[k] > tmax ? (int64_t)htot[k] : tmax;
    if (conc) {
        for (auto &a : c->aux)
            if (!a) GS_HIP(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        for (auto &e : c->aux_ev)
            if (!e) GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    int launched = 0;
    for (int k = 0; k < kJacClasses; ++k) {
        static const char *const kTrow[kJacClasses] = {"jac_trow0", "jac_trow1", "jac_trow2",
                                                      "jac_trow3", "jac_trow4"};
        static const char *const kTi[kJacClasses] = {"jac_ti0", "jac_ti1", "jac_ti2", "jac_ti3",
                                                    "jac_ti4"};
        const int64_t sz = htot[k] ? (int64_t)htot[k] : 1;
        auto *trow = (int32_t *)c->buf(conc ? kTrow[k] : "jac_trow").ensure(sizeof(int32_t) * (conc ? sz : tmax));
        auto *ti = (int32_t *)c->buf(conc ? kTi[k] : "jac_ti").ensure(sizeof(int32_t) * (conc ? sz : tmax));
        const bool giant = k == kJacBitmap;
        const int64_t ntot = (int64_t)htot[k], ngiant = giant ? (int64_t)htot[kJacClasses] : 0;
        if (!ntot) continue;
        int32_t *tslot = giant ? (int32_t *)c->buf("jac_tslot").ensure(sizeof(int32_t) * ntot)
                               : nullptr;
        int32_t *grow = giant ? (int32_t *)c->buf("jac_grow").ensure(sizeof(int32_t) * ngiant)
                              : nullptr;
        if (!cached) {
            GS_HIP(hipMemsetAsync(cnt + nr, 0, sizeof(int64_t), st));
            GS_HIP(hipMemsetAsync(gfl + nr, 0, sizeof(int64_t), st));
            k_jac_mask<<<grid_for(nr, 256, 16384), 256, 0, st>>>(cls, ntask, r0, r1, k, cnt,
                                                                 giant ? gfl : nullptr);
            exclusive_scan_i64(c, cnt, off, nr + 1);
            if (giant) exclusive_scan_i64(c, gfl, goff, nr + 1);
            k_jac_emit<<<grid_for(nr, 256, 16384), 256, 0, st>>>(cls, ntask, off, giant ? goff : nullptr,
                                                                 r0, r1, k, trow, ti, tslot, grow);
        }
        GS_HIP(hipGetLastError());
        GS_CHECK(ntot <= INT32_MAX, GS_EUNSUPPORTED, "too many Jaccard tasks (%lld)", (long long)ntot);
        // every emitted task is this part's (only its rows were planned)
        const int64_t tlo = 0, thi = ntot;
        const unsigned nb = (unsigned)(thi - tlo);
        if (k < kJacBitmap && !nb) continue;
        // hash classes: on side stream k once the task lists are emitted
        hipStream_t hs = st;
        if (conc && k < kJacBitmap) {
            GS_HIP(hipEventRecord(c->aux_ev[k], st));
            GS_HIP(hipStreamWaitEvent(c->aux[k], c->aux_ev[k], 0));
            hs = c->aux[k];
            launched |= 1 << k;
        }
        JacQParams qp{};
        const bool q16 = k >= 1 && k <= 3 && ((GS_JAC_Q16 >> k) & 1) &&
                         jac_qparams(n, k == 1 ? 16384 : 32768, qp);
        // test hook: a smaller largest distance, so the overflow path runs
        if (const char *e = q16 ? getenv("GSPARSE_JAC_QDMAX") : nullptr)
            if (atoi(e) >= 0 && (uint32_t)atoi(e) < qp.dmax) qp.dmax = (uint32_t)atoi(e);
        if (k == 0) {
            k_jac_hash<2048><<<nb, 256, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, sk);
        } else if (q16 && k == 1) {
            k_jac_hashq<16384, 512, 4><<<nb, 512, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, qp, sk);
        } else if (q16) {
            k_jac_hashq<32768, 1024, 8><<<nb, 1024, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, qp, sk);
        } else if (k == 1) {
            k_jac_hash<8192><<<nb, 512, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, sk);
        } else if (k == 2) {
            k_jac_hash<16384><<<nb, 1024, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, sk);
        } else if (k == 3) {
            k_jac_hash<32768><<<nb, 1024, 0, hs>>>(ip, ix, ntask, trow, ti, tlo, sk);
        } else {
            // bitmaps in batches of rows (<= 1 GiB of bits at a time); the batches' task
            // ranges are part of the kept plan
            const int64_t words = (n + 31) / 32;
            int64_t per = ((int64_t)1 << 30) / (4 * words);
            if (per < 1) per = 1;
            if (!cached) {
                std::vector<int32_t> hrow(ngiant);
                GS_HIP(hipMemcpyAsync(hrow.data(), grow, sizeof(int32_t) * ngiant,
                                      hipMemcpyDeviceToHost, st));
                GS_HIP(hipStreamSynchronize(st));
                for (int64_t g0 = 0; g0 < ngiant; g0 += per) {
                    const int64_t g1 = g0 + per < ngiant ? g0 + per : ngiant;
                    // task range of rows hrow[g0 .. g1): tasks are in row order
                    int64_t tb[2];
                    GS_HIP(hipMemcpyAsync(&tb[0], off + (hrow[g0] - r0), 8, hipMemcpyDeviceToHost, st));
                    if (g1 < ngiant)
                        GS_HIP(hipMemcpyAsync(&tb[1], off + (hrow[g1] - r0), 8, hipMemcpyDeviceToHost, st));
                    GS_HIP(hipStreamSynchronize(st));
                    if (g1 >= ngiant) tb[1] = ntot;
                    // this part's tasks only
                    if (tb[0] < tlo) tb[0] = tlo;
                    if (tb[1] > thi) tb[1] = thi;
                    c->jac_plan_bm.push_back({g0, g1, tb[0], tb[1]});
                }
            }
            for (const auto &bb : c->jac_plan_bm) {
                const int64_t g0 = bb[0], g1 = bb[1];
                const int64_t tb[2] = {bb[2], bb[3]};
                if (tb[1] <= tb[0]) continue;
                auto *bm = (uint32_t *)c->buf("jac_bitmap").ensure(sizeof(uint32_t) * words * (g1 - g0));
                GS_HIP(hipMemsetAsync(bm, 0, sizeof(uint32_t) * words * (g1 - g0), st));
                k_jac_bitmap_build<<<dim3(64, (unsigned)(g1 - g0)), 256, 0, st>>>(
                    ip, ix, grow, (int32_t)g0, words, bm);
                if (tb[1] > tb[0])
                    k_jac_bitmap<<<(unsigned)(tb[1] - tb[0]), 1024, 0, st>>>(
                        ip, ix, ntask, trow, ti, tslot, tb[0], (int32_t)g0, words, bm, sk);
                GS_HIP(hipGetLastError());
            }
        }
        GS_HIP(hipGetLastError());
    }
    // join the side streams back into the context stream
    for (int k = 0; k < kJacBitmap; ++k)
        if (launched & (1 << k)) {
            GS_HIP(hipEventRecord(c->aux_ev[k], c->aux[k]));
            GS_HIP(hipStreamWaitEvent(st, c->aux_ev[k], 0));
        }
    if (!cached && conc) c->jac_plan_key = pkey;
    prof_end(c, t0, counts ? "common_neighbors" : "jaccard", algo);
}

// gs_jaccard_from_counts: every part's counts -> the Jaccard score of every entry
void jaccard_from_counts(gs_ctx *c, int P, const uint32_t *cc, int64_t stride, double *out) {
    Graph &g = c->g;
    const int64_t nnz = g.nnz;
    if (!nnz) return;
    const JacShares &sh = jaccard_shares(c, P);
    for (int r = 0; r < P; ++r)
        GS_CHECK(sh.O(r + 1) - sh.O(r) <= stride, GS_EINDEX,
                 "part %d holds %lld owner pairs, more than the stride %lld", r,
                 (long long)(sh.O(r + 1) - sh.O(r)), (long long)stride);
    auto *dcut = (int64_t *)c->buf("jac_cutdev").ensure(sizeof(int64_t) * sh.cuts.size());
    GS_HIP(hipMemcpyAsync(dcut, sh.cuts.data(), sizeof(int64_t) * sh.cuts.size(),
                          hipMemcpyHostToDevice, c->stream));
    hipEvent_t t0 = prof_begin(c);
    const int64_t nown = sh.O(P);
    if (nnz < (int64_t)INT32_MAX) {
        // per owner pair: position, reverse position, d_u + d_v, the count (4 B each) in;
        // both entries (8 B each) out
        k_jac_scatter_owners<<<grid_for(nown, 256, 65536), 256, 0, c->stream>>>(
            c->buf("jac_opos").as<int32_t>(), c->buf("jac_orev").as<int32_t>(),
            c->buf("jac_osum").as<int32_t>(), dcut, P, cc, stride, nown, out);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jaccard_scatter", 32.0 * (double)nown);
    } else {
        k_jac_from_counts<<<grid_for(nnz, 256, 65536), 256, 0, c->stream>>>(
            g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.rows.as<int32_t>(), g.tpos.as<int64_t>(),
            c->buf("jac_opre").as<int64_t>(), dcut, P, cc, stride, nnz, out);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jaccard_scatter", 48.0 * (double)nnz + 8.0 * (double)nown);
    }
    // the host copy of cuts must outlive the async H2D copy: it lives in the cache
}

}  // namespace gs
