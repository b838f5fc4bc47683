// gs_rng.hip -- R = default_rng(seed).standard_normal((m, k)) on the device,
// bit-identical to NumPy (metrics.py:232,272), then Y = B @ (R / sqrt(k)).
//
// The stream is sequential (a normal consumes a variable number of PCG64
// draws), so it is parsed in parallel in three passes over blocks of
// kZigBlock draws, one thread per block, each block jumping straight to its
// first draw with the LCG jump-ahead:
//   scan : parse the block from offset 0, and from every other possible
//          entry offset e < 64 until that parse merges into the offset-0
//          attempt chain -> (normals produced, exit offset) per entry;
//   link : entry(t+1) = exit_t(entry(t)); nearly every block exits the same
//          way from every entry, so links resolve in parallel and only the
//          rare entry-dependent blocks are chained by one thread;
//   emit : exclusive scan of the selected counts -> first normal index of
//          each block; re-parse from the true entry and store the normals.
#include "gs_internal.hpp"
#include "gs_ziggurat.hpp"

namespace gs {

static constexpr int kZigEntries = 64;

struct ZigTables {
    int32_t *cnt;     // [nblk][64] normals produced from entry e
    uint8_t *ext;     // [nblk][64] exit offset into the next block from entry e
    uint8_t *prefc;   // [nblk][64] normals produced before chain position p (offset-0 parse)
    uint8_t *uniform; // [nblk] all entries exit the same way
    int32_t *entry;   // [nblk]
    int64_t *sel;     // [nblk] count for the resolved entry
    int64_t *base;    // [nblk] first normal index
    int32_t *pending; // [nblk] blocks whose entry needs the sequential link
    int32_t *flags;   // [0]: #pending, [1]: overflow
};

__global__ void __launch_bounds__(64) k_zig_scan(u128 s0, u128 inc, int64_t nblk, int kZigBlock, ZigTables T) {
    int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (t >= nblk) return;
    const u128 st = pcg_advance(s0, inc, (uint64_t)t * kZigBlock);
    int32_t *cnt = T.cnt + t * kZigEntries;
    uint8_t *ext = T.ext + t * kZigEntries;
    uint8_t *prefc = T.prefc + t * kZigEntries;
    Pcg64 g{st, inc};
    uint64_t mask = 0;
    int pos = 0, count = 0;
    bool prod;
    double v;
    while (pos < kZigBlock) {
        if (pos < kZigEntries) {
            mask |= 1ull << pos;
            prefc[pos] = (uint8_t)count;
        }
        int used = zig_attempt<true>(g, &prod, &v);
        count += prod ? 1 : 0;
        pos += used;
    }
    const int exit0 = pos - kZigBlock;
    const int count0 = count;
    if (exit0 >= kZigEntries) atomicOr(&T.flags[1], 1);
    bool uni = true;
    for (int e = 0; e < kZigEntries; ++e) {
        int ce, xe;
        if ((mask >> e) & 1ull) {
            ce = count0 - prefc[e];
            xe = exit0;
        } else {
            Pcg64 h{st, inc};
            for (int i = 0; i < e; ++i) (void)h.next();
            int p = e, c = 0;
            bool merged = false;
            while (p < kZigBlock) {
                if (p < kZigEntries && ((mask >> p) & 1ull)) {
                    merged = true;
                    break;
                }
                int used = zig_attempt<true>(h, &prod, &v);
                c += prod ? 1 : 0;
                p += used;
            }
            if (merged) {
                ce = c + count0 - prefc[p];
                xe = exit0;
            } else {
                ce = c;
                xe = p - kZigBlock;
                if (xe >= kZigEntries) atomicOr(&T.flags[1], 1);
            }
        }
        cnt[e] = ce;
        ext[e] = (uint8_t)(xe < kZigEntries ? xe : kZigEntries - 1);
        uni = uni && (xe == exit0);
    }
    T.uniform[t] = uni ? 1 : 0;
}

__global__ void k_zig_link(int64_t nblk, ZigTables T) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nblk;
         t += (int64_t)gridDim.x * blockDim.x) {
        if (t == 0) {
            T.entry[0] = 0;
        } else if (T.uniform[t - 1]) {
            T.entry[t] = T.ext[(t - 1) * kZigEntries];
        } else {
            T.entry[t] = -1;
            int q = atomicAdd(&T.flags[0], 1);
            T.pending[q] = (int32_t)t;
        }
    }
}

// one thread: chain the entry-dependent links in block order
__global__ void k_zig_link_seq(ZigTables T) {
    int np = T.flags[0];
    for (int i = 1; i < np; ++i) {  // insertion sort (np is ~0)
        int32_t x = T.pending[i];
        int j = i - 1;
        while (j >= 0 && T.pending[j] > x) {
            T.pending[j + 1] = T.pending[j];
            --j;
        }
        T.pending[j + 1] = x;
    }
    for (int i = 0; i < np; ++i) {
        int32_t t = T.pending[i];
        int32_t ep = T.entry[t - 1];
        T.entry[t] = T.ext[(int64_t)(t - 1) * kZigEntries + ep];
    }
}

__global__ void k_zig_select(int64_t nblk, ZigTables T) {
    for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nblk;
         t += (int64_t)gridDim.x * blockDim.x)
        T.sel[t] = T.cnt[t * kZigEntries + T.entry[t]];
}

// one thread per span of ge consecutive parse blocks (1,024 draws): the parse from the
// span's first entry runs straight through the later blocks' entries (the stream is
// deterministic), so the normals come out in order from the span's first index.
// Normal idx is R[idx / k, idx % k] (row-major m x k, NumPy's order); only the
// columns [c0, c1) are stored, as an m x (c1 - c0) row-major block (a rank's JL
// columns: every rank parses the whole stream, each stores only its own slice)
__global__ void __launch_bounds__(64) k_zig_emit(u128 s0, u128 inc, int64_t nblk, int kZigBlock, int ge,
                                                 ZigTables T, int64_t need, int64_t k, int64_t c0,
                                                 int64_t c1, double *__restrict__ out) {
    const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t b0 = t * ge;
    if (b0 >= nblk) return;
    int64_t idx = T.base[b0];
    if (idx >= need) return;
    const int e = T.entry[b0];
    const int span = (int)((b0 + ge <= nblk ? ge : nblk - b0) * kZigBlock);
    Pcg64 g{pcg_advance(s0, inc, (uint64_t)b0 * kZigBlock + e), inc};
    int pos = e;
    bool prod;
    double v;
    const int64_t kc = c1 - c0;
    if (kc == k) {
        while (pos < span && idx < need) {
            pos += zig_attempt<true>(g, &prod, &v);
            if (prod) out[idx++] = v;
        }
        return;
    }
    int64_t row = idx / k, col = idx - row * k;  // one division per span, then counters
    while (pos < span && idx < need) {
        pos += zig_attempt<true>(g, &prod, &v);
        if (prod) {
            if (col >= c0 && col < c1) out[row * kc + (col - c0)] = v;
            ++idx;
            if (++col == k) {
                col = 0;
                ++row;
            }
        }
    }
}

}  // namespace gs

using namespace gs;

extern "C" int gs_er_project_pcg64_cols(gs_ctx *c, uint64_t state_hi, uint64_t state_lo,
                                        uint64_t inc_hi, uint64_t inc_lo, double sqrt_k,
                                        int64_t col0, int64_t col1) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.k > 0, GS_ESTATE, "gs_er_prepare first");
        GS_CHECK(er.proj_next == 0, GS_ESTATE, "projection already started");
        GS_CHECK(0 <= col0 && col0 < col1 && col1 <= er.k, GS_EINVAL, "bad column range [%lld, %lld) of %lld",
                 (long long)col0, (long long)col1, (long long)er.k);
        GS_HIP(hipSetDevice(c->device));
        hipStream_t s = c->stream;
        const int64_t need = er.m * er.k;
        er.proj_c0 = col0;
        er.proj_c1 = col1;
        if (need == 0) return;
        const u128 s0 = ((u128)state_hi << 64) | state_lo;
        const u128 inc = ((u128)inc_hi << 64) | inc_lo;
        double *raw = (double *)er.rawbuf.ensure(sizeof(double) * (size_t)er.m * (size_t)(col1 - col0));
        hipEvent_t t0 = prof_begin(c);
        // draws per parse block: 256 while that still leaves few waves per SIMD (Roman:
        // 344 k scan threads instead of 86 k; the scan 1.37 -> 0.91 ms), 1,024 for long
        // streams, where the per-block tables (384 B per block) would otherwise add a
        // fifth to the bytes written.  The emit always walks 1,024-draw spans (256-draw
        // spans made its scattered stores slower: 0.63 -> 1.07 ms)
        int kZigBlock = need < ((int64_t)1 << 29) ? 256 : 1024;
        if (const char *e = getenv("GSPARSE_ZIG_BLOCK")) {
            const int v = atoi(e);
            if (v == 256 || v == 512 || v == 1024) kZigBlock = v;
        }
        // NumPy's ziggurat consumes 1.022 draws per normal on average (measured,
        // 2e6 normals); start with 4% headroom so one attempt suffices
        int64_t draws = need + need / 25 + 4 * (int64_t)kZigBlock;
        // a stream already parsed with this state, length and block size: the draw count
        // known to suffice (the parse is deterministic), so no host check is needed
        const std::vector<uint64_t> zkey = {state_hi, state_lo, inc_hi, inc_lo, (uint64_t)need,
                                            (uint64_t)kZigBlock};
        const bool known = zkey == c->zig_key;
        if (known) draws = c->zig_draws;
        for (int attempt = 0; attempt < 8; ++attempt) {
            int64_t nblk = (draws + kZigBlock - 1) / kZigBlock;
            ZigTables T;
            T.cnt = (int32_t *)c->buf("zig_cnt").ensure(sizeof(int32_t) * nblk * kZigEntries);
            T.ext = (uint8_t *)c->buf("zig_ext").ensure(nblk * kZigEntries);
            T.prefc = (uint8_t *)c->buf("zig_prefc").ensure(nblk * kZigEntries);
            T.uniform = (uint8_t *)c->buf("zig_uni").ensure(nblk);
            T.entry = (int32_t *)c->buf("zig_entry").ensure(sizeof(int32_t) * nblk);
            T.sel = (int64_t *)c->buf("zig_sel").ensure(sizeof(int64_t) * nblk);
            T.base = (int64_t *)c->buf("zig_base").ensure(sizeof(int64_t) * nblk);
            T.pending = (int32_t *)c->buf("zig_pending").ensure(sizeof(int32_t) * nblk);
            T.flags = (int32_t *)c->buf("zig_flags").ensure(64);
            GS_HIP(hipMemsetAsync(T.flags, 0, 64, s));
            k_zig_scan<<<(unsigned)((nblk + 63) / 64), 64, 0, s>>>(s0, inc, nblk, kZigBlock, T);
            k_zig_link<<<grid_for(nblk, 256, 4096), 256, 0, s>>>(nblk, T);
            k_zig_link_seq<<<1, 1, 0, s>>>(T);
            k_zig_select<<<grid_for(nblk, 256, 4096), 256, 0, s>>>(nblk, T);
            exclusive_scan_i64(c, T.sel, T.base, nblk);
            if (!known) {
                int64_t last[2];
                int32_t fl[2];
                GS_HIP(hipMemcpyAsync(&last[0], T.base + nblk - 1, 8, hipMemcpyDeviceToHost, s));
                GS_HIP(hipMemcpyAsync(&last[1], T.sel + nblk - 1, 8, hipMemcpyDeviceToHost, s));
                GS_HIP(hipMemcpyAsync(fl, T.flags, 8, hipMemcpyDeviceToHost, s));
                GS_HIP(hipStreamSynchronize(s));
                GS_CHECK(!fl[1], GS_EUNSUPPORTED,
                         "a ziggurat attempt crossed more than %d draws of a block boundary",
                         kZigEntries);
                if (last[0] + last[1] < need) {
                    draws = draws + draws / 4;
                    continue;
                }
                c->zig_key = zkey;
                c->zig_draws = draws;
            }
            const int ge = 1024 / kZigBlock;  // emit spans of 1,024 draws (fewer, longer store streams)
            const int64_t nspan = (nblk + ge - 1) / ge;
            k_zig_emit<<<(unsigned)((nspan + 63) / 64), 64, 0, s>>>(s0, inc, nblk, kZigBlock, ge, T, need,
                                                                    er.k, col0, col1, raw);
            GS_HIP(hipGetLastError());
            prof_end(c, t0, "er_rng", 8.0 * (double)er.m * (double)(col1 - col0));
            // Y[:, col0:col1] = B @ (R[:, col0:col1] / sqrt(k)) over all m rows, straight
            // from the device buffer
            project_rows(c, 0, er.m, raw, col1 - col0, col0, col1, sqrt_k);
            return;
        }
        GS_CHECK(false, GS_EHIP, "ziggurat draw estimate failed to converge");
    });
}

extern "C" int gs_er_project_pcg64(gs_ctx *c, uint64_t state_hi, uint64_t state_lo,
                                   uint64_t inc_hi, uint64_t inc_lo, double sqrt_k) {
    if (!c) return gs_er_project_pcg64_cols(c, state_hi, state_lo, inc_hi, inc_lo, sqrt_k, 0, 1);
    return gs_er_project_pcg64_cols(c, state_hi, state_lo, inc_hi, inc_lo, sqrt_k, 0, c->er.k);
}
