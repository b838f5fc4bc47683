// gs_graph.hip -- canonical CSR on the device.
//
// Replaces GraphSparsifier.__init__ (core.py:70-74):
//   sp.csr_matrix((np.ones(E), (ei[0], ei[1])), shape=(n, n))
// i.e. COO -> CSR with duplicates summed (data = multiplicity) and column
// indices sorted.  Here: 64-bit keys row*n+col, rocPRIM radix sort, run-length
// encode, row histogram + scan.  Layout in HBM: indptr int64[n+1],
// indices int32[nnz], data f64[nnz], rows int32[nnz] (row of each entry, so
// edge-parallel kernels need no search).
#include "gs_internal.hpp"

namespace gs {

static int bits_for(uint64_t v) {
    int b = 0;
    while (b < 64 && (v >> b)) ++b;
    return b < 1 ? 1 : b;
}

__global__ void k_make_keys(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                            int64_t E, int64_t n, uint64_t *__restrict__ keys,
                            int *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = src[i], d = dst[i];
        if (s < 0 || s >= n || d < 0 || d >= n) {
            atomicOr(bad, 1);
            s = 0;
            d = 0;
        }
        keys[i] = (uint64_t)s * (uint64_t)n + (uint64_t)d;
    }
}

__global__ void k_head_flags(const uint64_t *__restrict__ keys, int64_t E,
                             int64_t *__restrict__ flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x)
        flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

__global__ void k_compact_unique(const uint64_t *__restrict__ keys, const int64_t *__restrict__ flag,
                                 const int64_t *__restrict__ pos, int64_t E, int64_t n,
                                 int32_t *__restrict__ indices, int32_t *__restrict__ rows,
                                 int64_t *__restrict__ start) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (flag[i]) {
            int64_t j = pos[i];
            uint64_t k = keys[i];
            indices[j] = (int32_t)(k % (uint64_t)n);
            rows[j] = (int32_t)(k / (uint64_t)n);
            start[j] = i;
        }
    }
}

__global__ void k_counts(const int64_t *__restrict__ start, int64_t nnz, int64_t E,
                         double *__restrict__ data) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nnz;
         j += (int64_t)gridDim.x * blockDim.x) {
        int64_t e = (j + 1 < nnz) ? start[j + 1] : E;
        data[j] = (double)(e - start[j]);
    }
}

__global__ void k_row_hist(const int32_t *__restrict__ rows, int64_t nnz,
                           unsigned long long *__restrict__ cnt) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nnz;
         j += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&cnt[rows[j]], 1ull);
}

__global__ void k_rows_from_indptr(const int64_t *__restrict__ indptr, int64_t n,
                                   int32_t *__restrict__ rows) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        for (int64_t e = indptr[i]; e < indptr[i + 1]; ++e) rows[e] = (int32_t)i;
}

__global__ void k_fill_f64(double *p, int64_t n, double v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// Validate a caller-provided CSR: sorted, unique, in range.
__global__ void k_check_csr(const int64_t *__restrict__ indptr, const int32_t *__restrict__ idx,
                            int64_t n, int *__restrict__ bad) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t a = indptr[i], b = indptr[i + 1];
        if (b < a) { atomicOr(bad, 1); continue; }
        for (int64_t e = a; e < b; ++e) {
            int32_t v = idx[e];
            if (v < 0 || v >= n) atomicOr(bad, 2);
            if (e > a && idx[e - 1] >= v) atomicOr(bad, 4);
        }
    }
}

// transpose keys: col*n + row, payload = CSR position
__global__ void k_tkeys(const int32_t *__restrict__ rows, const int32_t *__restrict__ idx,
                        int64_t nnz, int64_t n, uint64_t *__restrict__ keys,
                        int64_t *__restrict__ pos) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nnz;
         j += (int64_t)gridDim.x * blockDim.x) {
        keys[j] = (uint64_t)idx[j] * (uint64_t)n + (uint64_t)rows[j];
        pos[j] = j;
    }
}

__global__ void k_tsplit(const uint64_t *__restrict__ keys, int64_t nnz, int64_t n,
                         int32_t *__restrict__ tidx, const int32_t *__restrict__ idx,
                         const int32_t *__restrict__ rows, int *__restrict__ asym) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < nnz;
         j += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[j];
        int32_t r = (int32_t)(k % (uint64_t)n);  // source row -> transposed column
        int32_t c = (int32_t)(k / (uint64_t)n);
        tidx[j] = r;
        // symmetric iff the transposed pattern equals the CSR pattern entry for entry
        if (r != idx[j] || c != rows[j]) atomicOr(asym, 1);
    }
}

// Canonical edge list (the loader's to_undirected + coalesce): keys of both
// directions, dropped entries (self-loops when asked) keyed n*n so the sort
// puts them last; sorted unique keys -> (row, col) int64.
__global__ void k_pair_keys(const int64_t *__restrict__ src, const int64_t *__restrict__ dst,
                            int64_t E, int64_t n, int both, int drop_loops,
                            uint64_t *__restrict__ keys, int *__restrict__ bad) {
    const uint64_t un = (uint64_t)n, drop = un * un;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = src[i], d = dst[i];
        if (s < 0 || s >= n || d < 0 || d >= n) {
            atomicOr(bad, 1);
            s = d = 0;
        }
        const bool gone = drop_loops && s == d;
        keys[i] = gone ? drop : (uint64_t)s * un + (uint64_t)d;
        if (both) keys[E + i] = gone ? drop : (uint64_t)d * un + (uint64_t)s;
    }
}

__global__ void k_compact_pairs(const uint64_t *__restrict__ keys, const int64_t *__restrict__ flag,
                                const int64_t *__restrict__ pos, int64_t E, int64_t n,
                                int64_t *__restrict__ row, int64_t *__restrict__ col) {
    const uint64_t un = (uint64_t)n;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < E;
         i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t k = keys[i];
        if (flag[i] && k < un * un) {
            row[pos[i]] = (int64_t)(k / un);
            col[pos[i]] = (int64_t)(k % un);
        }
    }
}

static void build_indptr_from_rows(gs_ctx *c) {
    Graph &g = c->g;
    int64_t n = g.n, nnz = g.nnz;
    int64_t *ip = (int64_t *)g.indptr.ensure(sizeof(int64_t) * (n + 1));
    unsigned long long *cnt = (unsigned long long *)c->scratch[0].ensure(sizeof(int64_t) * (n + 1));
    GS_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (n + 1), c->stream));
    if (nnz)
        k_row_hist<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(g.rows.as<int32_t>(), nnz, cnt);
    exclusive_scan_i64(c, (const int64_t *)cnt, ip, n + 1);
}

static void reset_derived(gs_ctx *c) {
    c->g.has_transpose = false;
    c->er = ErState{};  // buffers are released lazily below
}

static void finish_graph(gs_ctx *c) {
    Graph &g = c->g;
    ++g.epoch;
    g.has_transpose = false;
    g.symmetric = 0;
    // Drop any ER state bound to the old graph.
    DevBuf *eb[] = {&c->er.edge_id, &c->er.bptr, &c->er.bcol, &c->er.bsgn, &c->er.bcur,
                    &c->er.lp,      &c->er.li,   &c->er.lv,   &c->er.X,    &c->er.Rr,
                    &c->er.P0,      &c->er.P1,   &c->er.Q,    &c->er.colstate,
                    &c->er.acc,     &c->er.iters, &c->er.rawbuf};
    for (auto *b : eb) b->release();
    c->er = ErState{};
    ensure_transpose(c);
}

void ensure_transpose(gs_ctx *c) {
    Graph &g = c->g;
    if (g.has_transpose) return;
    int64_t n = g.n, nnz = g.nnz;
    g.tptr.ensure(sizeof(int64_t) * (n + 1));
    g.tidx.ensure(sizeof(int32_t) * (nnz ? nnz : 1));
    g.tpos.ensure(sizeof(int64_t) * (nnz ? nnz : 1));
    int *flag = (int *)c->scratch[1].ensure(64);
    GS_HIP(hipMemsetAsync(flag, 0, sizeof(int), c->stream));
    if (nnz) {
        uint64_t *keys = (uint64_t *)c->scratch[2].ensure(sizeof(uint64_t) * nnz);
        k_tkeys<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(
            g.rows.as<int32_t>(), g.indices.as<int32_t>(), nnz, n, keys, g.tpos.as<int64_t>());
        sort_pairs_u64_i64(c, keys, g.tpos.as<int64_t>(), nnz, bits_for((uint64_t)n * n));
        k_tsplit<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(
            keys, nnz, n, g.tidx.as<int32_t>(), g.indices.as<int32_t>(), g.rows.as<int32_t>(), flag);
        // in-degree histogram -> tptr
        unsigned long long *cnt =
            (unsigned long long *)c->scratch[0].ensure(sizeof(int64_t) * (n + 1));
        GS_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (n + 1), c->stream));
        k_row_hist<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(g.indices.as<int32_t>(), nnz,
                                                                    cnt);
        exclusive_scan_i64(c, (const int64_t *)cnt, g.tptr.as<int64_t>(), n + 1);
    } else {
        GS_HIP(hipMemsetAsync(g.tptr.ptr, 0, sizeof(int64_t) * (n + 1), c->stream));
    }
    int asym = 0;
    GS_HIP(hipMemcpyAsync(&asym, flag, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    GS_HIP(hipStreamSynchronize(c->stream));
    g.symmetric = asym ? 0 : 1;
    g.has_transpose = true;
}

}  // namespace gs

using namespace gs;

extern "C" {

int gs_graph_from_edge_index(gs_ctx *c, int64_t n, int64_t E, const int64_t *src,
                             const int64_t *dst, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(n >= 0 && E >= 0, GS_EINVAL, "negative n/E");
        GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31 nodes");
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        g.n = n;
        const int64_t *dsrc = (const int64_t *)to_device(c, c->inbuf, src, sizeof(int64_t) * E, loc);
        const int64_t *ddst = (const int64_t *)to_device(c, c->inbuf2, dst, sizeof(int64_t) * E, loc);
        int *bad = (int *)c->scratch[1].ensure(64);
        GS_HIP(hipMemsetAsync(bad, 0, sizeof(int), c->stream));
        int64_t nnz = 0;
        if (E > 0) {
            uint64_t *keys = (uint64_t *)c->scratch[2].ensure(sizeof(uint64_t) * E);
            k_make_keys<<<grid_for(E, 256, 8192), 256, 0, c->stream>>>(dsrc, ddst, E, n, keys, bad);
            int hbad = 0;
            GS_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
            GS_HIP(hipStreamSynchronize(c->stream));
            GS_CHECK(!hbad, GS_EINVAL, "edge_index entry out of range [0, %lld)", (long long)n);
            sort_keys_u64(c, keys, E, bits_for((uint64_t)n * (uint64_t)n));
            int64_t *flag = (int64_t *)c->scratch[0].ensure(sizeof(int64_t) * E);
            int64_t *pos = (int64_t *)c->scratch[1].ensure(sizeof(int64_t) * E + 64);
            k_head_flags<<<grid_for(E, 256, 8192), 256, 0, c->stream>>>(keys, E, flag);
            exclusive_scan_i64(c, flag, pos, E);
            int64_t last[2];
            GS_HIP(hipMemcpyAsync(&last[0], pos + E - 1, sizeof(int64_t), hipMemcpyDeviceToHost,
                                  c->stream));
            GS_HIP(hipMemcpyAsync(&last[1], flag + E - 1, sizeof(int64_t), hipMemcpyDeviceToHost,
                                  c->stream));
            GS_HIP(hipStreamSynchronize(c->stream));
            nnz = last[0] + last[1];
            g.indices.ensure(sizeof(int32_t) * (nnz + kIxPad));
            g.rows.ensure(sizeof(int32_t) * nnz);
            g.data.ensure(sizeof(double) * nnz);
            int64_t *start = (int64_t *)c->scratch[3].ensure(sizeof(int64_t) * nnz);
            k_compact_unique<<<grid_for(E, 256, 8192), 256, 0, c->stream>>>(
                keys, flag, pos, E, n, g.indices.as<int32_t>(), g.rows.as<int32_t>(), start);
            k_counts<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(start, nnz, E,
                                                                      g.data.as<double>());
        }
        g.nnz = nnz;
        build_indptr_from_rows(c);
        finish_graph(c);
    });
}

int gs_graph_from_csr(gs_ctx *c, int64_t n, int64_t nnz, const int64_t *indptr,
                      const int32_t *indices, const double *data, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(n >= 0 && nnz >= 0, GS_EINVAL, "negative n/nnz");
        GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31 nodes");
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        g.n = n;
        g.nnz = nnz;
        int64_t *ip = (int64_t *)g.indptr.ensure(sizeof(int64_t) * (n + 1));
        g.indices.ensure(sizeof(int32_t) * (nnz + kIxPad));
        g.data.ensure(sizeof(double) * (nnz ? nnz : 1));
        g.rows.ensure(sizeof(int32_t) * (nnz ? nnz : 1));
        GS_HIP(hipMemcpyAsync(ip, indptr, sizeof(int64_t) * (n + 1),
                              loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                              c->stream));
        if (nnz) {
            GS_HIP(hipMemcpyAsync(g.indices.ptr, indices, sizeof(int32_t) * nnz,
                                  loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                                  c->stream));
            if (data)
                GS_HIP(hipMemcpyAsync(g.data.ptr, data, sizeof(double) * nnz,
                                      loc == GS_DEVICE ? hipMemcpyDeviceToDevice
                                                       : hipMemcpyHostToDevice,
                                      c->stream));
            else
                k_fill_f64<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(g.data.as<double>(), nnz,
                                                                            1.0);
        }
        int *bad = (int *)c->scratch[1].ensure(64);
        GS_HIP(hipMemsetAsync(bad, 0, sizeof(int), c->stream));
        if (n)
            k_check_csr<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(ip, g.indices.as<int32_t>(), n,
                                                                       bad);
        int hbad = 0;
        int64_t last = 0;
        GS_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipMemcpyAsync(&last, ip + n, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        GS_CHECK(last == nnz, GS_EINVAL, "indptr[n]=%lld != nnz=%lld", (long long)last,
                 (long long)nnz);
        GS_CHECK(!(hbad & 3), GS_EINVAL, "CSR indices out of range or indptr not monotone");
        GS_CHECK(!(hbad & 4), GS_EUNSUPPORTED,
                 "CSR rows must have sorted, duplicate-free column indices (canonical format)");
        if (n)
            k_rows_from_indptr<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(ip, n,
                                                                              g.rows.as<int32_t>());
        finish_graph(c);
    });
}

int gs_coalesce_edges(gs_ctx *c, int64_t n, int64_t E, const int64_t *src, const int64_t *dst,
                      int undirected, int remove_self_loops, int64_t *out_src, int64_t *out_dst,
                      int64_t *out_E, int loc) {
    return guard([&] {
        GS_CHECK(c && out_E, GS_EINVAL, "null context/out_E");
        GS_CHECK(n >= 0 && E >= 0, GS_EINVAL, "negative n/E");
        GS_CHECK(n < (int64_t(1) << 31), GS_EUNSUPPORTED, "n >= 2^31 nodes");
        GS_HIP(hipSetDevice(c->device));
        const int64_t cap = *out_E, M = undirected ? 2 * E : E;
        *out_E = 0;
        if (E == 0) return;
        const int64_t *dsrc = (const int64_t *)to_device(c, c->inbuf, src, sizeof(int64_t) * E, loc);
        const int64_t *ddst = (const int64_t *)to_device(c, c->inbuf2, dst, sizeof(int64_t) * E, loc);
        int *bad = (int *)c->scratch[1].ensure(64);
        GS_HIP(hipMemsetAsync(bad, 0, sizeof(int), c->stream));
        uint64_t *keys = (uint64_t *)c->scratch[2].ensure(sizeof(uint64_t) * M);
        k_pair_keys<<<grid_for(E, 256, 8192), 256, 0, c->stream>>>(
            dsrc, ddst, E, n, undirected ? 1 : 0, remove_self_loops ? 1 : 0, keys, bad);
        int hbad = 0;
        GS_HIP(hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        GS_CHECK(!hbad, GS_EINVAL, "edge_index entry out of range [0, %lld)", (long long)n);
        const uint64_t un = (uint64_t)n;
        sort_keys_u64(c, keys, M, bits_for(un * un));
        int64_t *flag = (int64_t *)c->scratch[0].ensure(sizeof(int64_t) * M);
        int64_t *pos = (int64_t *)c->scratch[1].ensure(sizeof(int64_t) * M + 64);
        k_head_flags<<<grid_for(M, 256, 8192), 256, 0, c->stream>>>(keys, M, flag);
        exclusive_scan_i64(c, flag, pos, M);
        int64_t last[2];
        uint64_t lastkey = 0;
        GS_HIP(hipMemcpyAsync(&last[0], pos + M - 1, sizeof(int64_t), hipMemcpyDeviceToHost,
                              c->stream));
        GS_HIP(hipMemcpyAsync(&last[1], flag + M - 1, sizeof(int64_t), hipMemcpyDeviceToHost,
                              c->stream));
        GS_HIP(hipMemcpyAsync(&lastkey, keys + M - 1, sizeof(uint64_t), hipMemcpyDeviceToHost,
                              c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        const int64_t m = last[0] + last[1] - (lastkey == un * un ? 1 : 0);
        GS_CHECK(m <= cap, GS_EINVAL, "output capacity %lld < %lld edges", (long long)cap,
                 (long long)m);
        if (m > 0) {
            int64_t *orow = (int64_t *)c->scratch[3].ensure(sizeof(int64_t) * 2 * m);
            k_compact_pairs<<<grid_for(M, 256, 8192), 256, 0, c->stream>>>(keys, flag, pos, M, n,
                                                                           orow, orow + m);
            hipMemcpyKind kind = loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
            GS_HIP(hipMemcpyAsync(out_src, orow, sizeof(int64_t) * m, kind, c->stream));
            GS_HIP(hipMemcpyAsync(out_dst, orow + m, sizeof(int64_t) * m, kind, c->stream));
            GS_HIP(hipStreamSynchronize(c->stream));
        }
        *out_E = m;
    });
}

int gs_graph_shape(gs_ctx *c, int64_t *n, int64_t *nnz, int *symmetric) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        if (n) *n = c->g.n;
        if (nnz) *nnz = c->g.nnz;
        if (symmetric) *symmetric = c->g.symmetric;
    });
}

int gs_graph_copy_csr(gs_ctx *c, int64_t *indptr, int32_t *indices, double *data, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        hipMemcpyKind kind = loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
        if (indptr)
            GS_HIP(hipMemcpyAsync(indptr, g.indptr.ptr, sizeof(int64_t) * (g.n + 1), kind, c->stream));
        if (indices && g.nnz)
            GS_HIP(hipMemcpyAsync(indices, g.indices.ptr, sizeof(int32_t) * g.nnz, kind, c->stream));
        if (data && g.nnz)
            GS_HIP(hipMemcpyAsync(data, g.data.ptr, sizeof(double) * g.nnz, kind, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

}  // extern "C"
