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

__global__ void k_fill_u8(uint8_t *p, int64_t n, uint8_t v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
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
        prof_end(c, t0, "topk", 9.0 * 8.0 * nnz + 8.0 * nnz + E);
        finish_out(c, mask, dm, E, m_loc);
        if (cut) *cut = hcut;
        if (n_beyond) *n_beyond = hbeyond;
        if (n_tied) *n_tied = htied;
    });
}
