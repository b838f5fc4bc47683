// gs_jsel.hip -- the global top-k of Jaccard-T (GraphSparsifier.sparsify, core.py:229-240)
// over N ranks without gathering the scores ("top-k alone: histogram
// all-reduce").
//
// Each rank holds the owner-pair counts of its row share (gs_jaccard_part_counts).  A
// pair's two CSR entries carry the same score (|N(u) ∩ N(v)| is symmetric and the
// reference's single fp64 division is the same for both), so the selection runs over the
// rank's pairs with multiplicity 2 (1 for a self-loop):
//   begin   score and order-preserving 64-bit key of every own pair, the 12-bit
//           histogram of the keys' top bits (weighted)        -> all-reduce (SUM)
//   step    pick the digit holding the cut's rank from the reduced histogram, then the
//           next 13-bit digit's histogram of the keys under the chosen prefix; five
//           digits (12 + 4 x 13 bits) give the cut key        -> all-reduce after each
//   result  the cut, the entries strictly beyond it and the tie block, as one GPU's
//           radix select gives them (every rank holds the same reduced histograms)
//   ties    (an ambiguous cut only) this rank's tied CSR positions -> all-gather
//   keep    a 2-bit keep code per own pair (bit 0 the owner entry, bit 1 its reverse
//           entry), four per byte; the tie block resolved as np.argsort(kind='stable')
//           resolves it (top: the highest positions; keep_lowest: the lowest)
//                                                              -> all-gather (E / 8 bytes)
//   mask    every rank's codes -> the whole CSR keep mask (a gather through a per-entry
//           code index cached per graph and part count)
// The mask is bit-identical to gs_topk_mask on the gathered scores (the device tie rule).
#include "gs_internal.hpp"

#include <map>
#include <mutex>

namespace gs {

static constexpr int kJselBins = 8192;
static constexpr int kJselPasses = 5;
__host__ __device__ constexpr int jsel_shift(int p) { return p == 0 ? 52 : 52 - 13 * p; }
__host__ __device__ constexpr int jsel_bits(int p) { return p == 0 ? 12 : 13; }

struct JselDev {
    unsigned long long prefix;  // chosen key bits
    unsigned long long rank;    // rank of the cut among the keys under the prefix (ascending)
    unsigned long long below;   // entries with keys below the prefix's bucket (all passes)
    unsigned long long eq;      // entries at the cut key (after the last pass)
    unsigned long long ntie;    // this rank's tied CSR positions (ties kernel)
};

struct JselHost {
    int part = -1, nparts = 0, pass = 0;
    int64_t npairs = 0, obase = 0, num_keep = 0, nnz = 0;
    int keep_lowest = 0;
    // slot table: (graph epoch, nparts, stride) it was built for
    std::vector<int64_t> slot_key;
};
static std::mutex g_jsel_mu;
static std::map<gs_ctx *, JselHost> g_jsel;

__device__ __forceinline__ uint64_t jsel_key(double x) {
    if (x == 0.0) x = 0.0;  // -0.0 -> +0.0 (Jaccard scores are >= 0 and never NaN)
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

static double jsel_key_value(uint64_t k) {
    uint64_t b = (k >> 63) ? (k & 0x7fffffffffffffffull) : ~k;
    double d;
    memcpy(&d, &b, 8);
    return d;
}

// own pair i (global owner index obase + i): score, key, weight
__global__ void k_jsel_keys(const uint32_t *__restrict__ cc, const int32_t *__restrict__ opos,
                            const int32_t *__restrict__ orev, const int32_t *__restrict__ osum,
                            int64_t obase, int64_t np, uint64_t *__restrict__ keys,
                            uint8_t *__restrict__ wt, double *__restrict__ scores) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t g = obase + i, cnt = cc[i];
        // k_jac_scatter_owners' value: fl(d_u + d_v) is exact, one fp64 division
        const double uni = (double)osum[g] - (double)cnt;
        const double val = uni > 0.0 ? (double)cnt / uni : 0.0;
        keys[i] = jsel_key(val);
        wt[i] = opos[g] == orev[g] ? 1 : 2;
        if (scores) scores[i] = val;
    }
}

// weighted histogram of digit p of the keys under the prefix (pass 0: every key)
__global__ void __launch_bounds__(256) k_jsel_hist(const uint64_t *__restrict__ keys,
                                                   const uint8_t *__restrict__ wt, int64_t np,
                                                   const JselDev *__restrict__ st, int pass,
                                                   unsigned long long *__restrict__ hist) {
    __shared__ unsigned int h[kJselBins];
    for (int i = threadIdx.x; i < kJselBins; i += 256) h[i] = 0;
    __syncthreads();
    const int shift = jsel_shift(pass), top = shift + jsel_bits(pass);
    const uint64_t hmask = top >= 64 ? 0ull : ~0ull << top;
    const uint64_t pre = st->prefix & hmask;
    const uint64_t dmask = (1ull << jsel_bits(pass)) - 1;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < np;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[i];
        if ((k & hmask) == pre) atomicAdd(&h[(k >> shift) & dmask], (unsigned int)wt[i]);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kJselBins; i += 256)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

// one workgroup: the digit of the reduced histogram that holds the cut's rank
__global__ void __launch_bounds__(256) k_jsel_pick(JselDev *st, const unsigned long long *__restrict__ hist,
                                                   int pass) {
    __shared__ unsigned long long part[256];
    const int t = threadIdx.x, nb = 1 << jsel_bits(pass), per = nb / 256;
    unsigned long long s = 0;
    for (int i = 0; i < per; ++i) s += hist[t * per + i];
    part[t] = s;
    __syncthreads();
    if (t == 0) {
        const unsigned long long r = st->rank;
        unsigned long long acc = 0;
        int b = 0;
        for (; b < 255 && r >= acc + part[b]; ++b) acc += part[b];
        int d = b * per;
        for (; d < b * per + per - 1 && r >= acc + hist[d]; ++d) acc += hist[d];
        st->rank = r - acc;
        st->below += acc;
        st->prefix |= (unsigned long long)d << jsel_shift(pass);
        if (pass == kJselPasses - 1) st->eq = hist[d];
    }
}

__global__ void k_jsel_ties(const uint64_t *__restrict__ keys, const int32_t *__restrict__ opos,
                            const int32_t *__restrict__ orev, int64_t obase, int64_t np,
                            JselDev *__restrict__ st, int64_t *__restrict__ pos) {
    const uint64_t cut = st->prefix;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t trips = (np + stride - 1) / stride;
    const int lane = threadIdx.x & 63;
    for (int64_t tr = 0, i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tr < trips; ++tr, i += stride) {
        const bool tie = i < np && keys[i] == cut;
        const int two = tie && opos[obase + i] != orev[obase + i] ? 1 : 0;
        const unsigned long long m = __ballot(tie), m2 = __ballot(two != 0);
        if (!m) continue;
        const int leader = __builtin_ctzll(m);
        unsigned long long base = 0;
        if (lane == leader) base = atomicAdd(&st->ntie, (unsigned long long)(__popcll(m) + __popcll(m2)));
        base = __shfl(base, leader, 64);
        const unsigned long long below = (1ull << lane) - 1ull;
        if (tie) {
            const unsigned long long p = base + __popcll(m & below) + __popcll(m2 & below);
            pos[p] = opos[obase + i];
            if (two) pos[p + 1] = orev[obase + i];
        }
    }
}

// rank of position x in the sorted tie block (every tied position is in it)
__device__ __forceinline__ int64_t jsel_tie_rank(const uint64_t *__restrict__ tall, int64_t ntie, uint64_t x) {
    int64_t lo = 0, hi = ntie;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (tall[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// mode 0: ties none kept, 1: all kept, 2: by rank in the sorted block.  Keep codes are
// 2 bits per pair (bit 0 the owner entry, bit 1 the reverse), four pairs per byte: one
// thread per byte, so no two threads share one
__device__ __forceinline__ uint32_t jsel_code(uint64_t k, uint64_t cut, int keep_lowest, int mode,
                                              const uint64_t *__restrict__ tall, int64_t ntie, int64_t need,
                                              int32_t pa, int32_t pb) {
    if (k != cut) return (keep_lowest ? k < cut : k > cut) ? 3u : 0u;
    if (mode != 2) return mode ? 3u : 0u;
    const int64_t ra = jsel_tie_rank(tall, ntie, (uint64_t)pa);
    const int64_t rb = jsel_tie_rank(tall, ntie, (uint64_t)pb);
    const bool ka = keep_lowest ? ra < need : ra >= ntie - need;
    const bool kb = keep_lowest ? rb < need : rb >= ntie - need;
    return (ka ? 1u : 0u) | (kb ? 2u : 0u);
}

__global__ void k_jsel_keep(const uint64_t *__restrict__ keys, const int32_t *__restrict__ opos,
                            const int32_t *__restrict__ orev, int64_t obase, int64_t np,
                            const JselDev *__restrict__ st, int keep_lowest, int mode,
                            const uint64_t *__restrict__ tall, int64_t ntie, int64_t need,
                            uint8_t *__restrict__ keep) {
    const uint64_t cut = st->prefix;
    const int64_t nb = (np + 3) >> 2;
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nb;
         q += (int64_t)gridDim.x * blockDim.x) {
        uint32_t b = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int64_t i = 4 * q + t;
            if (i < np)
                b |= jsel_code(keys[i], cut, keep_lowest, mode, tall, ntie, need, opos[obase + i],
                               orev[obase + i]) << (2 * t);
        }
        keep[q] = (uint8_t)b;
    }
}

// per CSR entry: the code index of its pair in the gathered buffer (part r's codes from
// r * 4 * stride, stride in bytes), bit 31 set for the pair's reverse entry
__global__ void k_jsel_slots(const int32_t *__restrict__ opos, const int32_t *__restrict__ orev,
                             const int64_t *__restrict__ O, int P, int64_t stride, int64_t nown,
                             uint32_t *__restrict__ slot) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nown;
         i += (int64_t)gridDim.x * blockDim.x) {
        int lo = 0, hi = P - 1;  // last part r with O[r] <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (O[mid] <= i) lo = mid;
            else hi = mid - 1;
        }
        const uint32_t s = (uint32_t)(4 * lo * stride + (i - O[lo]));
        slot[opos[i]] = s;
        if (orev[i] != opos[i]) slot[orev[i]] = s | 0x80000000u;
    }
}

// the gathered codes (~E / 8 bytes: 8 MB at R-MAT-22, mostly L2-resident) read by code index
__global__ void k_jsel_mask(const uint32_t *__restrict__ slot, const uint8_t *__restrict__ kall,
                            int64_t nnz, uint8_t *__restrict__ mask) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t s = slot[e], c = s & 0x7fffffffu;
        mask[e] = (kall[c >> 2] >> (2 * (c & 3) + (s >> 31))) & 1;
    }
}

void jsel_forget(gs_ctx *c) {
    std::lock_guard<std::mutex> lk(g_jsel_mu);
    g_jsel.erase(c);
}

}  // namespace gs

using namespace gs;

static JselHost &jsel_host(gs_ctx *c) {
    std::lock_guard<std::mutex> lk(g_jsel_mu);
    return g_jsel[c];
}

static void jsel_check_graph(gs_ctx *c, int nparts) {
    GS_CHECK(c, GS_EINVAL, "null context");
    GS_CHECK(nparts >= 1 && nparts <= 4096, GS_EINVAL, "bad part count %d", nparts);
    GS_CHECK(c->g.has_transpose, GS_ESTATE, "no graph set");
    GS_CHECK(c->g.symmetric, GS_EUNSUPPORTED, "the owner-pair select needs a symmetric graph");
    GS_CHECK(c->g.nnz < (int64_t)INT32_MAX, GS_EUNSUPPORTED, "the owner-pair select needs nnz < 2^31");
}

extern "C" int gs_jsel_begin(gs_ctx *c, int part, int nparts, const uint32_t *counts, int c_loc,
                             int64_t num_keep, int keep_lowest, uint64_t *hist, double *scores,
                             int s_loc) {
    return guard([&] {
        jsel_check_graph(c, nparts);
        GS_CHECK(0 <= part && part < nparts, GS_EINVAL, "bad part %d of %d", part, nparts);
        GS_CHECK(hist, GS_EINVAL, "null histogram");
        GS_HIP(hipSetDevice(c->device));
        const int64_t nnz = c->g.nnz;
        GS_CHECK(0 < num_keep && num_keep < nnz, GS_EINVAL,
                 "num_keep %lld outside (0, %lld): nothing to select", (long long)num_keep, (long long)nnz);
        const JacShares &sh = jaccard_shares(c, nparts);
        JselHost &H = jsel_host(c);
        H.part = part;
        H.nparts = nparts;
        H.pass = 0;
        H.obase = sh.O(part);
        H.npairs = sh.O(part + 1) - sh.O(part);
        H.num_keep = num_keep;
        H.nnz = nnz;
        H.keep_lowest = keep_lowest ? 1 : 0;
        hipStream_t s = c->stream;
        const int64_t np = H.npairs;
        const uint32_t *dc = (const uint32_t *)to_device(c, c->inbuf, counts, sizeof(uint32_t) * (np ? np : 1), c_loc);
        auto *keys = (uint64_t *)c->buf("jsel_keys").ensure(sizeof(uint64_t) * (np ? np : 1));
        auto *wt = (uint8_t *)c->buf("jsel_wt").ensure(np ? np : 1);
        double *ds = scores ? (double *)out_device(c, c->outbuf, scores, sizeof(double) * (np ? np : 1), s_loc) : nullptr;
        auto *st = (JselDev *)c->buf("jsel_state").ensure(sizeof(JselDev));
        JselDev init{};
        init.rank = keep_lowest ? (unsigned long long)(num_keep - 1) : (unsigned long long)(nnz - num_keep);
        // stream-ordered upload from a host value that must outlive it: synchronised below
        GS_HIP(hipMemcpyAsync(st, &init, sizeof(JselDev), hipMemcpyHostToDevice, s));
        GS_HIP(hipMemsetAsync(hist, 0, sizeof(uint64_t) * kJselBins, s));
        hipEvent_t t0 = prof_begin(c);
        if (np) {
            k_jsel_keys<<<grid_for(np, 256, 65536), 256, 0, s>>>(dc, c->buf("jac_opos").as<int32_t>(),
                                                                c->buf("jac_orev").as<int32_t>(),
                                                                c->buf("jac_osum").as<int32_t>(), H.obase, np,
                                                                keys, wt, ds);
            k_jsel_hist<<<grid_for(np, 256, 1024), 256, 0, s>>>(keys, wt, np, st, 0,
                                                                (unsigned long long *)hist);
        }
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jsel_keys", 17.0 * (double)np);
        if (ds) finish_out(c, scores, ds, sizeof(double) * np, s_loc);
        GS_HIP(hipStreamSynchronize(s));  // `init` is on this frame
    });
}

extern "C" int gs_jsel_step(gs_ctx *c, uint64_t *hist, int *passes_left) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        JselHost &H = jsel_host(c);
        GS_CHECK(H.part >= 0, GS_ESTATE, "gs_jsel_begin first");
        GS_CHECK(H.pass < kJselPasses, GS_ESTATE, "all %d passes done", kJselPasses);
        GS_CHECK(hist, GS_EINVAL, "null histogram");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        auto *st = (JselDev *)c->buf("jsel_state").ptr;
        hipEvent_t t0 = prof_begin(c);
        k_jsel_pick<<<1, 256, 0, s>>>(st, (const unsigned long long *)hist, H.pass);
        ++H.pass;
        if (H.pass < kJselPasses) {
            GS_HIP(hipMemsetAsync(hist, 0, sizeof(uint64_t) * kJselBins, s));
            if (H.npairs)
                k_jsel_hist<<<grid_for(H.npairs, 256, 1024), 256, 0, s>>>(
                    c->buf("jsel_keys").as<uint64_t>(), c->buf("jsel_wt").as<uint8_t>(), H.npairs, st, H.pass,
                    (unsigned long long *)hist);
        }
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jsel_pass", 9.0 * (double)H.npairs);
        if (passes_left) *passes_left = kJselPasses - H.pass;
        sync_if_needed(c);  // hist (a device output) is complete on return
    });
}

extern "C" int gs_jsel_result(gs_ctx *c, double *cut, int64_t *n_beyond, int64_t *n_tied,
                              int64_t *my_tied) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        JselHost &H = jsel_host(c);
        GS_CHECK(H.part >= 0 && H.pass == kJselPasses, GS_ESTATE, "gs_jsel_step x %d first", kJselPasses);
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        auto *st = (JselDev *)c->buf("jsel_state").ptr;
        GS_HIP(hipMemsetAsync(&st->ntie, 0, 8, s));
        auto *pos = (int64_t *)c->buf("jsel_tpos").ensure(sizeof(int64_t) * 2 * (H.npairs ? H.npairs : 1));
        if (H.npairs)
            k_jsel_ties<<<grid_for(H.npairs, 256, 2048), 256, 0, s>>>(
                c->buf("jsel_keys").as<uint64_t>(), c->buf("jac_opos").as<int32_t>(), c->buf("jac_orev").as<int32_t>(),
                H.obase, H.npairs, st, pos);
        GS_HIP(hipGetLastError());
        JselDev h{};
        GS_HIP(hipMemcpyAsync(&h, st, sizeof(JselDev), hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
        const int64_t below = (int64_t)h.below, eq = (int64_t)h.eq;
        if (cut) *cut = jsel_key_value(h.prefix);
        if (n_beyond) *n_beyond = H.keep_lowest ? below : H.nnz - below - eq;
        if (n_tied) *n_tied = eq;
        if (my_tied) *my_tied = (int64_t)h.ntie;
    });
}

extern "C" int gs_jsel_tie_positions(gs_ctx *c, int64_t *pos, int64_t npos, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        JselHost &H = jsel_host(c);
        GS_CHECK(H.part >= 0 && H.pass == kJselPasses, GS_ESTATE, "gs_jsel_result first");
        GS_HIP(hipSetDevice(c->device));
        unsigned long long mine = 0;
        auto *st = (JselDev *)c->buf("jsel_state").ptr;
        GS_HIP(hipMemcpyAsync(&mine, &st->ntie, 8, hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        GS_CHECK(npos >= (int64_t)mine, GS_EINDEX, "pos holds %lld, this rank has %llu tied positions",
                 (long long)npos, mine);
        if (!mine) return;
        GS_CHECK(pos, GS_EINVAL, "null positions");
        GS_HIP(hipMemcpyAsync(pos, c->buf("jsel_tpos").ptr, 8 * mine,
                              loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

extern "C" int gs_jsel_keep(gs_ctx *c, const int64_t *tie_pos, int64_t ntie, int t_loc, int64_t need,
                            uint8_t *keep, int k_loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        JselHost &H = jsel_host(c);
        GS_CHECK(H.part >= 0 && H.pass == kJselPasses, GS_ESTATE, "gs_jsel_result first");
        GS_CHECK(ntie >= 0, GS_EINVAL, "negative tie count");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        const int mode = need <= 0 ? 0 : need >= ntie ? 1 : 2;
        uint64_t *tall = nullptr;
        if (mode == 2) {
            GS_CHECK(tie_pos, GS_EINVAL, "an ambiguous cut needs every rank's tied positions");
            tall = (uint64_t *)c->buf("jsel_tall").ensure(8 * ntie);
            GS_HIP(hipMemcpyAsync(tall, tie_pos, 8 * ntie,
                                  t_loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
            int eb = 1;
            while (eb < 64 && ((uint64_t)H.nnz >> eb)) ++eb;
            sort_keys_u64(c, tall, ntie, eb);
        }
        const int64_t np = H.npairs, nb = (np + 3) / 4;
        uint8_t *dk = (uint8_t *)out_device(c, c->outbuf, keep, nb ? nb : 1, k_loc);
        hipEvent_t t0 = prof_begin(c);
        if (np)
            k_jsel_keep<<<grid_for(nb, 256, 65536), 256, 0, s>>>(
                c->buf("jsel_keys").as<uint64_t>(), c->buf("jac_opos").as<int32_t>(), c->buf("jac_orev").as<int32_t>(),
                H.obase, np, (const JselDev *)c->buf("jsel_state").ptr, H.keep_lowest, mode, tall, ntie, need, dk);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jsel_keep", 16.25 * (double)np);
        finish_out(c, keep, dk, nb, k_loc);
        if (mode == 2 && t_loc != GS_DEVICE) GS_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int gs_jsel_mask(gs_ctx *c, int nparts, const uint8_t *keep_all, int64_t stride, int k_loc,
                            uint8_t *mask, int m_loc) {
    return guard([&] {
        jsel_check_graph(c, nparts);
        GS_CHECK(stride >= 0, GS_EINVAL, "negative stride");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        const JacShares &sh = jaccard_shares(c, nparts);
        for (int r = 0; r < nparts; ++r)
            GS_CHECK((sh.O(r + 1) - sh.O(r) + 3) / 4 <= stride, GS_EINDEX,
                     "part %d holds %lld owner pairs, more than the stride %lld bytes of codes hold", r,
                     (long long)(sh.O(r + 1) - sh.O(r)), (long long)stride);
        GS_CHECK(4 * (int64_t)nparts * stride < ((int64_t)1 << 31), GS_EUNSUPPORTED, "keep codes past 2^31");
        const int64_t nnz = c->g.nnz, nown = sh.O(nparts);
        JselHost &H = jsel_host(c);
        auto *slot = (uint32_t *)c->buf("jsel_slot").ensure(sizeof(uint32_t) * (nnz ? nnz : 1));
        const std::vector<int64_t> key = {c->g.epoch, nparts, stride, (int64_t)(uintptr_t)slot};
        if (H.slot_key != key) {
            auto *dcut = (int64_t *)c->buf("jsel_cuts").ensure(sizeof(int64_t) * sh.cuts.size());
            GS_HIP(hipMemcpyAsync(dcut, sh.cuts.data(), sizeof(int64_t) * sh.cuts.size(), hipMemcpyHostToDevice, s));
            if (nown)
                k_jsel_slots<<<grid_for(nown, 256, 65536), 256, 0, s>>>(
                    c->buf("jac_opos").as<int32_t>(), c->buf("jac_orev").as<int32_t>(), dcut + 2 * (nparts + 1),
                    nparts, stride, nown, slot);
            GS_HIP(hipGetLastError());
            H.slot_key = key;
        }
        const uint8_t *dk = (const uint8_t *)to_device(c, c->inbuf, keep_all, (size_t)(nparts * stride ? nparts * stride : 1), k_loc);
        uint8_t *dm = (uint8_t *)out_device(c, c->outbuf, mask, nnz ? nnz : 1, m_loc);
        hipEvent_t t0 = prof_begin(c);
        if (nnz) k_jsel_mask<<<grid_for(nnz, 256, 65536), 256, 0, s>>>(slot, dk, nnz, dm);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "jsel_mask", 5.25 * (double)nnz);
        finish_out(c, mask, dm, nnz, m_loc);
    });
}
