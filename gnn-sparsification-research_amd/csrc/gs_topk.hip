// gs_topk.hip -- global top-k edge mask (GraphSparsifier.sparsify,
// core.py:229-242) by MSB-first radix select over order-preserving 64-bit
// keys of the fp64 scores: 8 passes of an 8-bit LDS histogram (one read of
// the scores per pass, no sort), then one mask pass.  Ties at the cut are
// resolved as np.argsort(kind='stable') resolves them (top: the highest
// indices; keep_lowest: the lowest), with a device exclusive scan over the
// tie flags.  NaN orders last (np.sort), -0.0 == +0.0.
#include "gs_internal.hpp"

namespace gs {

__device__ __forceinline__ uint64_t order_key(double x) {
    if (x != x) return ~0ull;
    if (x == 0.0) x = 0.0;  // -0.0 -> +0.0
    uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

static double key_to_double(uint64_t k) {
    uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double d;
    memcpy(&d, &b, 8);
    return d;
}

struct SelState {
    unsigned long long prefix;  // selected high bits
    unsigned long long rank;    // remaining rank inside the prefix bucket
    unsigned long long hist[256];
};

__global__ void __launch_bounds__(256) k_hist(const double *__restrict__ s, int64_t nnz,
                                              SelState *__restrict__ st, int shift) {
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t prefix = st->prefix;
    const uint64_t hmask = (shift >= 56) ? 0ull : (~0ull << (shift + 8));
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = order_key(s[i]);
        if ((k & hmask) == (prefix & hmask)) atomicAdd(&h[(k >> shift) & 0xff], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&st->hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

__global__ void k_pick(SelState *st, int shift) {
    unsigned long long r = st->rank, acc = 0;
    int d = 0;
    for (; d < 256; ++d) {
        unsigned long long cnt = st->hist[d];
        if (r < acc + cnt) break;
        acc += cnt;
    }
    if (d == 256) d = 255;  // unreachable for a valid rank
    st->rank = r - acc;
    st->prefix |= (unsigned long long)d << shift;
    for (int i = 0; i < 256; ++i) st->hist[i] = 0;
}

__global__ void k_cut_counts(const double *__restrict__ s, int64_t nnz, const SelState *st,
                             int keep_lowest, unsigned long long *__restrict__ cnts,
                             int64_t *__restrict__ tie) {
    const uint64_t t = st->prefix;
    unsigned long long beyond = 0, eq = 0;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = order_key(s[i]);
        bool b = keep_lowest ? (k < t) : (k > t);
        beyond += b;
        eq += (k == t);
        tie[i] = (k == t) ? 1 : 0;
    }
    // wave reduce then one atomic per wave
    for (int off = 32; off > 0; off >>= 1) {
        beyond += __shfl_down(beyond, off, 64);
        eq += __shfl_down(eq, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&cnts[0], beyond);
        atomicAdd(&cnts[1], eq);
    }
}

__global__ void k_mask(const double *__restrict__ s, int64_t nnz, const SelState *st,
                       int keep_lowest, const int64_t *__restrict__ tiepos,
                       const unsigned long long *__restrict__ cnts, int64_t num_keep,
                       uint8_t *__restrict__ mask) {
    const uint64_t t = st->prefix;
    const int64_t beyond = (int64_t)cnts[0], ntied = (int64_t)cnts[1];
    const int64_t need = num_keep - beyond;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = order_key(s[i]);
        uint8_t m;
        if (k == t) {
            int64_t p = tiepos[i];
            m = keep_lowest ? (p < need) : (p >= ntied - need);
        } else {
            m = keep_lowest ? (k < t) : (k > t);
        }
        mask[i] = m;
    }
}

// ---- round 5: a 12-bit first pass, then the candidates only ----------------------
// Pass 1 histograms the keys' top 12 bits; the bucket holding the cut is picked on
// the device; pass 2 compacts that bucket's (key, index) pairs; the other 52 bits
// are selected on the candidates alone; one last pass over the scores writes the
// mask, and the tie block at the cut (its indices sorted) is resolved as
// np.argsort(kind='stable') resolves it.  Three reads of the scores instead of the
// nine reads and the per-element tie scan of the 8-bit form (kept as GSPARSE_TOPK=8).
struct Sel12 {
    unsigned long long hist[4096];
    unsigned long long rank;     // rank of the cut inside the candidates (ascending keys)
    unsigned long long prefix;   // selected key bits
    unsigned long long outside;  // keys strictly beyond the cut bucket (top: above it)
    unsigned long long ncand, nbeyond_c, ntied;
    unsigned long long chist[256];
};

__global__ void __launch_bounds__(256) k_hist12(const double *__restrict__ s, int64_t nnz,
                                                Sel12 *__restrict__ st) {
    __shared__ unsigned int h[4096];
    for (int i = threadIdx.x; i < 4096; i += 256) h[i] = 0;
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nnz;
         i += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&h[order_key(s[i]) >> 52], 1u);
    __syncthreads();
    for (int i = threadIdx.x; i < 4096; i += 256)
        if (h[i]) atomicAdd(&st->hist[i], (unsigned long long)h[i]);
}

// one workgroup of 256: bucket d holding rank r (ascending), the candidates' rank,
// the count beyond the bucket on the kept side
__global__ void __launch_bounds__(256) k_pick12(Sel12 *st, int keep_lowest) {
    __shared__ unsigned long long part[256];
    const int t = threadIdx.x;
    unsigned long long sum = 0;
    for (int i = 0; i < 16; ++i) sum += st->hist[t * 16 + i];
    part[t] = sum;
    __syncthreads();
    if (t == 0) {
        const unsigned long long r = st->rank;
        unsigned long long acc = 0, total = 0;
        for (int i = 0; i < 256; ++i) total += part[i];
        int b = 0;
        for (; b < 255 && r >= acc + part[b]; ++b) acc += part[b];
        int d = b * 16;
        for (; d < b * 16 + 15 && r >= acc + st->hist[d]; ++d) acc += st->hist[d];
        const unsigned long long c = st->hist[d];
        st->rank = r - acc;
        st->prefix = (unsigned long long)d << 52;
        st->ncand = c;
        st->outside = keep_lowest ? acc : total - acc - c;
        st->nbeyond_c = 0;
        st->ntied = 0;
        for (int i = 0; i < 256; ++i) st->chist[i] = 0;
    }
}

// one global atomic per wave and trip (the cut's bucket may hold millions of scores)
__device__ __forceinline__ unsigned long long wave_slot(bool take, unsigned long long *cnt) {
    const unsigned long long m = __ballot(take);
    if (!m) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(cnt, (unsigned long long)__popcll(m));
    base = __shfl(base, leader, 64);
    return base + (unsigned long long)__popcll(m & ((1ull << lane) - 1ull));
}

// block b compacts its range [b chunk, (b + 1) chunk) into the same range of ckey
// (slots from an LDS counter, one LDS atomic per wave and trip): no global counter --
// the cut's bucket may hold millions of scores (R-MAT-22: 7.7 M), and one global
// atomic per wave on a single address took 12 ms
__global__ void __launch_bounds__(256) k_compact12(const double *__restrict__ s, int64_t nnz, int64_t chunk,
                                                   const Sel12 *__restrict__ st, uint64_t *__restrict__ ckey,
                                                   unsigned int *__restrict__ bcount) {
    __shared__ unsigned int n_loc;
    if (threadIdx.x == 0) n_loc = 0;
    __syncthreads();
    const uint64_t d = st->prefix >> 52;
    const int64_t b0 = (int64_t)blockIdx.x * chunk;
    const int64_t b1 = b0 + chunk < nnz ? b0 + chunk : nnz;
    const int lane = threadIdx.x & 63;
    for (int64_t i0 = b0; i0 < b1; i0 += blockDim.x) {  // whole waves run every trip
        const int64_t i = i0 + threadIdx.x;
        const uint64_t k = i < b1 ? order_key(s[i]) : 0ull;
        const bool take = i < b1 && (k >> 52) == d;
        const unsigned long long m = __ballot(take);
        if (m) {
            const int leader = __builtin_ctzll(m);
            unsigned int base = 0;
            if (lane == leader) base = atomicAdd(&n_loc, (unsigned int)__popcll(m));
            base = __shfl(base, leader, 64);
            if (take) ckey[b0 + base + __popcll(m & ((1ull << lane) - 1ull))] = k;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) bcount[blockIdx.x] = n_loc;
}

// digit = bits [shift, shift + bits) of the candidates matching the prefix above it
// (block b: the candidates of region b, bcount[b] of them from b chunk)
__global__ void __launch_bounds__(256) k_chist(const uint64_t *__restrict__ ckey, const unsigned int *__restrict__ bcount,
                                               int64_t chunk, Sel12 *__restrict__ st, int shift, int bits) {
    __shared__ unsigned int h[256];
    h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t prefix = st->prefix;
    const uint64_t hmask = ~0ull << (shift + bits);
    const uint64_t dmask = (1ull << bits) - 1;
    const uint64_t *ck = ckey + (int64_t)blockIdx.x * chunk;
    const int64_t nc = bcount[blockIdx.x];
    for (int64_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const uint64_t k = ck[i];
        if ((k & hmask) == (prefix & hmask)) atomicAdd(&h[(k >> shift) & dmask], 1u);
    }
    __syncthreads();
    if (h[threadIdx.x]) atomicAdd(&st->chist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

__global__ void k_cpick(Sel12 *st, int shift) {
    unsigned long long r = st->rank, acc = 0;
    int d = 0;
    for (; d < 255; ++d) {
        const unsigned long long c = st->chist[d];
        if (r < acc + c) break;
        acc += c;
    }
    st->rank = r - acc;
    st->prefix |= (unsigned long long)d << shift;
    for (int i = 0; i < 256; ++i) st->chist[i] = 0;
}

// beyond / tied among the candidates (block b: region b)
__global__ void __launch_bounds__(256) k_ccount(const uint64_t *__restrict__ ckey, const unsigned int *__restrict__ bcount,
                                                int64_t chunk, Sel12 *__restrict__ st, int keep_lowest) {
    const uint64_t t = st->prefix;
    const uint64_t *ck = ckey + (int64_t)blockIdx.x * chunk;
    const int64_t nc = bcount[blockIdx.x];
    unsigned long long b = 0, e = 0;
    for (int64_t i = threadIdx.x; i < nc; i += blockDim.x) {
        const uint64_t k = ck[i];
        b += keep_lowest ? (k < t) : (k > t);
        e += k == t;
    }
    for (int off = 32; off > 0; off >>= 1) {
        b += __shfl_down(b, off, 64);
        e += __shfl_down(e, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        if (b) atomicAdd(&st->nbeyond_c, b);
        if (e) atomicAdd(&st->ntied, e);
    }
}

// mask of the strictly-beyond keys; the tie block's indices (unordered) collected
__global__ void k_mask12(const double *__restrict__ s, int64_t nnz, const Sel12 *__restrict__ st,
                         int keep_lowest, uint8_t *__restrict__ mask, unsigned long long *__restrict__ tcnt,
                         uint64_t *__restrict__ tidx) {
    const uint64_t t = st->prefix;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t trips = (nnz + stride - 1) / stride;
    for (int64_t tr = 0, i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tr < trips; ++tr, i += stride) {
        const uint64_t k = i < nnz ? order_key(s[i]) : 0ull;
        if (i < nnz) mask[i] = keep_lowest ? (k < t) : (k > t);
        const bool tie = i < nnz && k == t;
        const unsigned long long p = wave_slot(tie, tcnt);
        if (tie) tidx[p] = (uint64_t)i;
    }
}

// the tie block in ascending index order: top keeps its last `need`, keep_lowest its first
__global__ void k_tie_set(const uint64_t *__restrict__ tidx, int64_t ntied, int64_t need, int keep_lowest,
                          uint8_t *__restrict__ mask) {
    for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < ntied;
         p += (int64_t)gridDim.x * blockDim.x)
        if (keep_lowest ? p < need : p >= ntied - need) mask[tidx[p]] = 1;
}

__global__ void k_fill_u8(uint8_t *p, int64_t n, uint8_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// Per-node argmax of the incident columns (sparsify_degree_aware phase 1,
// core.py:415-428 with min_edges_per_node = 1): pick[u] = the column of the
// unique maximum, -1 if u has no column, -2 when np.argsort's order decides
// (several columns at the maximum, or a NaN score) -- the caller resolves
// those nodes with the reference's own call.
__global__ void k_seg_init(int64_t n, unsigned long long *__restrict__ mkey,
                           unsigned long long *__restrict__ cnt, unsigned long long *__restrict__ ncol,
                           int *__restrict__ nan, int64_t *__restrict__ idx) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        mkey[u] = 0ull;
        cnt[u] = 0ull;
        ncol[u] = 0ull;
        nan[u] = 0;
        idx[u] = -1;
    }
}

__global__ void k_seg_max(const double *__restrict__ s, const int64_t *__restrict__ src, int64_t E,
                          unsigned long long *__restrict__ mkey, unsigned long long *__restrict__ ncol,
                          int *__restrict__ nan) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[i];
        const double x = s[i];
        atomicAdd(&ncol[u], 1ull);
        if (x != x) atomicOr(&nan[u], 1);
        else atomicMax(&mkey[u], (unsigned long long)order_key(x));
    }
}

__global__ void k_seg_count(const double *__restrict__ s, const int64_t *__restrict__ src,
                            int64_t E, const unsigned long long *__restrict__ mkey,
                            unsigned long long *__restrict__ cnt, int64_t *__restrict__ idx) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = src[i];
        const double x = s[i];
        if (x == x && order_key(x) == mkey[u]) {
            atomicAdd(&cnt[u], 1ull);
            idx[u] = i;  // the only writer when the maximum is unique
        }
    }
}

__global__ void k_seg_pick(int64_t n, const unsigned long long *__restrict__ cnt,
                           const unsigned long long *__restrict__ ncol, const int *__restrict__ nan,
                           const int64_t *__restrict__ idx, int64_t *__restrict__ pick) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x)
        pick[u] = ncol[u] == 0 ? -1 : (nan[u] || cnt[u] != 1) ? -2 : idx[u];
}

__global__ void k_seg_check(const int64_t *__restrict__ src, int64_t E, int64_t n,
                            int *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        if (src[i] < 0 || src[i] >= n) atomicOr(bad, 1);
}

}  // namespace gs

using namespace gs;

extern "C" int gs_topk_mask(gs_ctx *c, const double *scores, int s_loc, int64_t nnz, int64_t E,
                            int64_t num_keep, int keep_lowest, uint8_t *mask, int m_loc,
                            double *cut, int64_t *n_beyond, int64_t *n_tied) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(nnz >= 0 && E >= nnz, GS_EINVAL, "need 0 <= nnz <= E (nnz=%lld, E=%lld)",
                 (long long)nnz, (long long)E);
        GS_HIP(hipSetDevice(c->device));
        const double *ds = (const double *)to_device(c, c->inbuf, scores, sizeof(double) * nnz, s_loc);
        uint8_t *dm = (uint8_t *)out_device(c, c->outbuf, mask, E ? E : 1, m_loc);
        if (E) GS_HIP(hipMemsetAsync(dm, 0, E, c->stream));
        double hcut = __builtin_nan("");
        int64_t hbeyond = 0, htied = 0;
        bool all = (!keep_lowest && num_keep <= 0) || num_keep >= nnz;  // idx[-0:] quirk
        bool none = keep_lowest && num_keep <= 0;
        hipEvent_t t0 = prof_begin(c);
        if (nnz == 0 || none) {
            // nothing kept
        } else if (all) {
            k_fill_u8<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(dm, nnz, 1);
            hbeyond = nnz;
        } else if (!getenv("GSPARSE_TOPK") || atoi(getenv("GSPARSE_TOPK")) != 8) {
            hipStream_t s = c->stream;
            Sel12 *st = (Sel12 *)c->buf("topk_sel12").ensure(sizeof(Sel12) + 64);
            unsigned long long *cnt = (unsigned long long *)((char *)st + sizeof(Sel12));
            uint64_t *ckey = (uint64_t *)c->buf("topk_ckey").ensure(sizeof(uint64_t) * nnz);
            GS_HIP(hipMemsetAsync(st, 0, sizeof(Sel12) + 64, s));
            const unsigned long long r0 = keep_lowest ? (unsigned long long)(num_keep - 1)
                                                      : (unsigned long long)(nnz - num_keep);
            GS_HIP(hipMemcpyAsync(&st->rank, &r0, 8, hipMemcpyHostToDevice, s));
            // the rank's host source must outlive the async copy: wait for it below
            const unsigned g = grid_for(nnz, 256, 1024);
            k_hist12<<<g, 256, 0, s>>>(ds, nnz, st);
            k_pick12<<<1, 256, 0, s>>>(st, keep_lowest);
            // regions: one per compaction workgroup
            const int64_t nreg = std::max<int64_t>(1, std::min<int64_t>(2048, nnz / 8192 + 1));
            const int64_t chunk = (nnz + nreg - 1) / nreg;
            auto *bcount = (unsigned int *)c->buf("topk_bcount").ensure(sizeof(unsigned int) * nreg);
            k_compact12<<<(unsigned)nreg, 256, 0, s>>>(ds, nnz, chunk, st, ckey, bcount);
            // the other 52 bits: six 8-bit digits (bits 51..4), then the last 4 bits
            for (int shift = 44; shift >= -4; shift -= 8) {
                const int sh = shift < 0 ? 0 : shift, bits = shift < 0 ? 4 : 8;
                k_chist<<<(unsigned)nreg, 256, 0, s>>>(ckey, bcount, chunk, st, sh, bits);
                k_cpick<<<1, 1, 0, s>>>(st, sh);
            }
            k_ccount<<<(unsigned)nreg, 256, 0, s>>>(ckey, bcount, chunk, st, keep_lowest);
            uint64_t *tidx = (uint64_t *)c->buf("topk_tidx").ensure(sizeof(uint64_t) * nnz);
            GS_HIP(hipMemsetAsync(cnt, 0, 8, s));
            k_mask12<<<grid_for(nnz, 256, 2048), 256, 0, s>>>(ds, nnz, st, keep_lowest, dm, cnt, tidx);
            GS_HIP(hipGetLastError());
            unsigned long long hs[3];
            uint64_t key;
            GS_HIP(hipMemcpyAsync(hs, &st->outside, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipMemcpyAsync(hs + 1, &st->nbeyond_c, 16, hipMemcpyDeviceToHost, s));
            GS_HIP(hipMemcpyAsync(&key, &st->prefix, 8, hipMemcpyDeviceToHost, s));
            GS_HIP(hipStreamSynchronize(s));
            if (getenv("GSPARSE_TOPK_DEBUG")) {
                unsigned long long nc = 0;
                GS_HIP(hipMemcpy(&nc, &st->ncand, 8, hipMemcpyDeviceToHost));
                fprintf(stderr, "[topk] nnz=%lld candidates=%llu tied=%llu\n", (long long)nnz, nc, hs[2]);
            }
            hbeyond = (int64_t)(hs[0] + hs[1]);
            htied = (int64_t)hs[2];
            hcut = key_to_double(key);
            const int64_t need = num_keep - hbeyond;
            if (need > 0 && htied > 0) {
                if (need < htied) {
                    int eb = 1;
                    while (eb < 64 && ((uint64_t)nnz >> eb)) ++eb;
                    sort_keys_u64(c, tidx, htied, eb);
                }
                k_tie_set<<<grid_for(htied, 256, 8192), 256, 0, s>>>(tidx, htied, need, keep_lowest, dm);
                GS_HIP(hipGetLastError());
            }
        } else {
            SelState *st = (SelState *)c->scratch[0].ensure(sizeof(SelState) + 64);
            unsigned long long *cnts = (unsigned long long *)((char *)st + sizeof(SelState));
            int64_t *tie = (int64_t *)c->scratch[1].ensure(sizeof(int64_t) * nnz);
            int64_t *tiepos = (int64_t *)c->scratch[2].ensure(sizeof(int64_t) * nnz);
            SelState init{};
            init.prefix = 0;
            init.rank = keep_lowest ? (unsigned long long)(num_keep - 1)
                                    : (unsigned long long)(nnz - num_keep);
            GS_HIP(hipMemcpyAsync(st, &init, sizeof(SelState), hipMemcpyHostToDevice, c->stream));
            GS_HIP(hipMemsetAsync(cnts, 0, 16, c->stream));
            unsigned g = grid_for(nnz, 256, 2048);
            for (int shift = 56; shift >= 0; shift -= 8) {
                k_hist<<<g, 256, 0, c->stream>>>(ds, nnz, st, shift);
                k_pick<<<1, 1, 0, c->stream>>>(st, shift);
            }
            k_cut_counts<<<g, 256, 0, c->stream>>>(ds, nnz, st, keep_lowest, cnts, tie);
            exclusive_scan_i64(c, tie, tiepos, nnz);
            k_mask<<<g, 256, 0, c->stream>>>(ds, nnz, st, keep_lowest, tiepos, cnts, num_keep, dm);
            GS_HIP(hipGetLastError());
            unsigned long long hc[2];
            uint64_t key;
            GS_HIP(hipMemcpyAsync(hc, cnts, 16, hipMemcpyDeviceToHost, c->stream));
            GS_HIP(hipMemcpyAsync(&key, &st->prefix, 8, hipMemcpyDeviceToHost, c->stream));
            GS_HIP(hipStreamSynchronize(c->stream));
            hbeyond = (int64_t)hc[0];
            htied = (int64_t)hc[1];
            hcut = key_to_double(key);
        }
        prof_end(c, t0, "topk", 3.0 * 8.0 * nnz + E);  // three reads of the scores, the mask
        finish_out(c, mask, dm, E, m_loc);
        if (cut) *cut = hcut;
        if (n_beyond) *n_beyond = hbeyond;
        if (n_tied) *n_tied = htied;
    });
}

extern "C" int gs_segment_argmax(gs_ctx *c, const double *scores, int s_loc, int64_t nscores,
                                 const int64_t *src, int src_loc, int64_t E, int64_t n,
                                 int64_t *pick, int pick_loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(n >= 0 && E >= 0, GS_EINVAL, "negative n/E");
        GS_CHECK(E <= nscores, GS_EINVAL,
                 "index %lld is out of bounds for axis 0 with size %lld (scores are per CSR "
                 "entry, columns per edge_index)", (long long)(E ? E - 1 : 0), (long long)nscores);
        GS_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        const double *ds = (const double *)to_device(c, c->buf("seg_s"), scores,
                                                     sizeof(double) * (E ? E : 1), s_loc);
        const int64_t *dsrc = (const int64_t *)to_device(c, c->buf("seg_src"), src,
                                                         sizeof(int64_t) * (E ? E : 1), src_loc);
        int64_t *dpick = (int64_t *)out_device(c, c->buf("seg_pick"), pick,
                                               sizeof(int64_t) * (n ? n : 1), pick_loc);
        auto *mkey = (unsigned long long *)c->buf("seg_mkey").ensure(8 * (n ? n : 1));
        auto *cnt = (unsigned long long *)c->buf("seg_cnt").ensure(8 * (n ? n : 1));
        auto *ncol = (unsigned long long *)c->buf("seg_ncol").ensure(8 * (n ? n : 1));
        auto *nan = (int *)c->buf("seg_nan").ensure(4 * (n ? n : 1) + 64);
        int *bad = nan + (n ? n : 1);
        auto *idx = (int64_t *)c->buf("seg_idx").ensure(8 * (n ? n : 1));
        GS_HIP(hipMemsetAsync(bad, 0, 4, st));
        if (E) k_seg_check<<<grid_for(E, 256, 8192), 256, 0, st>>>(dsrc, E, n, bad);
        int hbad = 0;
        GS_HIP(hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));
        GS_CHECK(!hbad, GS_EINVAL, "edge_index source out of range [0, %lld)", (long long)n);
        hipEvent_t t0 = prof_begin(c);
        if (n) k_seg_init<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, mkey, cnt, ncol, nan, idx);
        if (E) {
            k_seg_max<<<grid_for(E, 256, 8192), 256, 0, st>>>(ds, dsrc, E, mkey, ncol, nan);
            k_seg_count<<<grid_for(E, 256, 8192), 256, 0, st>>>(ds, dsrc, E, mkey, cnt, idx);
        }
        if (n) k_seg_pick<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, cnt, ncol, nan, idx, dpick);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "segment_argmax", 8.0 * 3 * (double)E + 8.0 * (double)n);
        finish_out(c, pick, dpick, sizeof(int64_t) * n, pick_loc);
    });
}
