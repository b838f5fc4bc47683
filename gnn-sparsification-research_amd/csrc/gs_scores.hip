// gs_scores.hip -- neighbour-intersection and feature scorers.
//
// Jaccard   metrics.py:17-64   |out(u) ∩ in(v)| / (deg u + deg v - inter)
// AA        metrics.py:67-121  sum_{w in out(u) ∩ out(v), w descending} c_w*c_w
// degree    core.py:167-172    deg[u] * deg[v], deg = multiplicity row sums
// FeatCos   metrics.py:301-358 pairwise-summed cosine of normalised rows
//
// One thread per CSR entry (edge).  The intersection walks the shorter list
// and gallops (exponential + binary search) through the longer one when the
// lengths are skewed, else it merges.  Integer counts are exact; the single
// fp64 divide is IEEE (correctly rounded) on gfx950, so Jaccard is
// bit-identical to the reference.  AA folds matches from the HIGH end so the
// fp64 accumulation order equals SciPy csr_matmat's (see oracle.c).
#include "gs_internal.hpp"
#include "gs_pairwise.hpp"

#include <cstdlib>
#include <cstring>

namespace gs {

// first index in b[lo..hi) with b[i] >= x (b sorted ascending)
__device__ __forceinline__ int64_t lower_bound_gallop(const int32_t *__restrict__ b, int64_t lo,
                                                      int64_t hi, int32_t x) {
    int64_t step = 1, probe = lo;
    while (probe < hi && b[probe] < x) {
        lo = probe + 1;
        probe = lo + step;
        step <<= 1;
    }
    if (probe > hi) probe = hi;
    while (lo < probe) {
        int64_t mid = (lo + probe) >> 1;
        if (b[mid] < x) lo = mid + 1;
        else probe = mid;
    }
    return lo;
}

__device__ __forceinline__ int64_t intersect_count(const int32_t *__restrict__ a, int64_t la,
                                                   const int32_t *__restrict__ b, int64_t lb) {
    if (la > lb) {
        const int32_t *t = a; a = b; b = t;
        int64_t tl = la; la = lb; lb = tl;
    }
    int64_t cnt = 0;
    if (la == 0) return 0;
    if (lb > 8 * la) {
        int64_t pos = 0;
        for (int64_t i = 0; i < la && pos < lb; ++i) {
            int32_t x = a[i];
            pos = lower_bound_gallop(b, pos, lb, x);
            if (pos < lb && b[pos] == x) { ++cnt; ++pos; }
        }
        return cnt;
    }
    int64_t i = 0, j = 0;
    while (i < la && j < lb) {
        int32_t x = a[i], y = b[j];
        cnt += (x == y);
        i += (x <= y);
        j += (y <= x);
    }
    return cnt;
}

__global__ void __launch_bounds__(256) k_jaccard(const int64_t *__restrict__ ip,
                                                 const int32_t *__restrict__ ix,
                                                 const int32_t *__restrict__ rows,
                                                 const int64_t *__restrict__ tp,
                                                 const int32_t *__restrict__ ti, int64_t e0,
                                                 int64_t e1, double *__restrict__ out) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x) {
        int32_t u = rows[e], v = ix[e];
        int64_t au = ip[u], du = ip[u + 1] - au;
        int64_t bv = tp[v], lv = tp[v + 1] - bv;
        int64_t inter = intersect_count(ix + au, du, ti + bv, lv);
        double dv = (double)(ip[v + 1] - ip[v]);
        double uni = (double)du + dv - (double)inter;
        out[e - e0] = uni > 0.0 ? (double)inter / uni : 0.0;
    }
}

// AA: iterate the shorter out-list from its END, search in the longer one.
__global__ void __launch_bounds__(256) k_adamic_adar(const int64_t *__restrict__ ip,
                                                     const int32_t *__restrict__ ix,
                                                     const int32_t *__restrict__ rows,
                                                     const double *__restrict__ c, int64_t e0,
                                                     int64_t e1, double *__restrict__ out) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x) {
        int32_t u = rows[e], v = ix[e];
        const int32_t *a = ix + ip[u];
        int64_t la = ip[u + 1] - ip[u];
        const int32_t *b = ix + ip[v];
        int64_t lb = ip[v + 1] - ip[v];
        if (la > lb) {
            const int32_t *t = a; a = b; b = t;
            int64_t tl = la; la = lb; lb = tl;
        }
        double s = 0.0;
        if (lb > 8 * la) {
            int64_t hi = lb;  // search window b[0..hi)
            for (int64_t i = la - 1; i >= 0 && hi > 0; --i) {
                int32_t x = a[i];
                int64_t lo = 0, h = hi;
                while (lo < h) {
                    int64_t mid = (lo + h) >> 1;
                    if (b[mid] < x) lo = mid + 1;
                    else h = mid;
                }
                if (lo < hi && b[lo] == x) {
                    double cw = c[x];
                    double p = cw * cw;
                    s = s + p;
                }
                hi = lo;
            }
        } else {
            int64_t i = la - 1, j = lb - 1;
            while (i >= 0 && j >= 0) {
                int32_t x = a[i], y = b[j];
                if (x == y) {
                    double cw = c[x];
                    double p = cw * cw;
                    s = s + p;
                    --i;
                    --j;
                } else if (x > y) {
                    --i;
                } else {
                    --j;
                }
            }
        }
        out[e - e0] = s;
    }
}

__global__ void k_row_sums(const int64_t *__restrict__ ip, const double *__restrict__ data,
                           int64_t n, double *__restrict__ deg) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e) s = s + data[e];
        deg[i] = s;
    }
}

__global__ void k_degree(const int32_t *__restrict__ rows, const int32_t *__restrict__ ix,
                         const double *__restrict__ deg, int64_t e0, int64_t e1,
                         double *__restrict__ out) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x)
        out[e - e0] = deg[rows[e]] * deg[ix[e]];
}

// FeatCos step 1: xn[i,:] = x[i,:] / max(sqrt(0 + pw(x*x)), T(1e-10))
template <class T>
__global__ void k_normalise(const T *__restrict__ x, int64_t n, int64_t f, T *__restrict__ xn) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const T *r = x + i * f;
        T ss = T(0) + pw_sum<T>(f, [&](int64_t k) {
                   T v = r[k];
                   return v * v;
               });
        T nrm = sizeof(T) == 4 ? (T)__builtin_sqrtf((float)ss) : (T)__builtin_sqrt((double)ss);
        const T fl = (T)1e-10;
        if (!(nrm >= fl)) nrm = (nrm != nrm) ? nrm : fl;  // np.maximum keeps NaN
        T *o = xn + i * f;
        for (int64_t k = 0; k < f; ++k) o[k] = r[k] / nrm;
    }
}

// FeatCos step 2: s = max(0 + pw(xn_u * xn_v), 0) in T, widened to f64.
template <class T>
__global__ void k_cosine(const int32_t *__restrict__ rows, const int32_t *__restrict__ ix,
                         const T *__restrict__ xn, int64_t f, int64_t e0, int64_t e1,
                         double *__restrict__ out) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x) {
        const T *a = xn + (int64_t)rows[e] * f;
        const T *b = xn + (int64_t)ix[e] * f;
        T s = T(0) + pw_sum<T>(f, [&](int64_t k) { return a[k] * b[k]; });
        if (!(s >= T(0))) s = (s != s) ? s : T(0);
        out[e - e0] = (double)s;
    }
}

static void check_range(gs_ctx *c, int64_t e0, int64_t e1) {
    GS_CHECK(c, GS_EINVAL, "null context");
    GS_CHECK(0 <= e0 && e0 <= e1 && e1 <= c->g.nnz, GS_EINVAL,
             "edge range [%lld, %lld) outside [0, %lld)", (long long)e0, (long long)e1,
             (long long)c->g.nnz);
}

template <class T>
static void feature_cosine(gs_ctx *c, const T *x, int64_t f, int x_loc, int64_t e0, int64_t e1,
                           double *out, int loc) {
    check_range(c, e0, e1);
    GS_CHECK(f >= 0, GS_EINVAL, "negative feature dim");
    GS_HIP(hipSetDevice(c->device));
    Graph &g = c->g;
    int64_t n = g.n, cnt = e1 - e0;
    const T *dx = (const T *)to_device(c, c->inbuf, x, sizeof(T) * n * f, x_loc);
    T *xn = (T *)c->scratch[0].ensure(sizeof(T) * (n * f > 0 ? n * f : 1));
    double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * cnt, loc);
    if (n) {
        hipEvent_t t0 = prof_begin(c);
        k_normalise<T><<<grid_for(n, 64), 64, 0, c->stream>>>(dx, n, f, xn);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "featcos_normalise", 2.0 * sizeof(T) * n * f);
    }
    if (cnt) {
        hipEvent_t t0 = prof_begin(c);
        k_cosine<T><<<grid_for(cnt, 64), 64, 0, c->stream>>>(g.rows.as<int32_t>(),
                                                            g.indices.as<int32_t>(), xn, f, e0,
                                                            e1, dout);
        GS_HIP(hipGetLastError());
        prof_end(c, t0, "featcos_edges", (2.0 * sizeof(T) * f + 16.0) * cnt);
    }
    finish_out(c, out, dout, sizeof(double) * cnt, loc);
}

}  // namespace gs

using namespace gs;

extern "C" {

int gs_jaccard(gs_ctx *c, int64_t e0, int64_t e1, double *out, int loc) {
    return guard([&] {
        check_range(c, e0, e1);
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        int64_t cnt = e1 - e0;
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * cnt, loc);
        const char *mode = getenv("GSPARSE_JACCARD");
        const bool merge_only = mode && strcmp(mode, "merge") == 0;
        if (cnt && g.symmetric && e0 == 0 && e1 == g.nnz && !merge_only) {
            jaccard_symmetric(c, dout, 0, 1);  // owner-side hash/bitmap probing, both entries written
        } else if (cnt) {
            const int64_t *tp = g.symmetric ? g.indptr.as<int64_t>() : g.tptr.as<int64_t>();
            const int32_t *ti = g.symmetric ? g.indices.as<int32_t>() : g.tidx.as<int32_t>();
            hipEvent_t t0 = prof_begin(c);
            k_jaccard<<<grid_for(cnt, 256), 256, 0, c->stream>>>(g.indptr.as<int64_t>(),
                                                                g.indices.as<int32_t>(),
                                                                g.rows.as<int32_t>(), tp, ti, e0,
                                                                e1, dout);
            GS_HIP(hipGetLastError());
            prof_end(c, t0, "jaccard", 0.0);
        }
        finish_out(c, out, dout, sizeof(double) * cnt, loc);
    });
}

int gs_jaccard_part(gs_ctx *c, int part, int nparts, double *out, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(nparts >= 1 && nparts <= 4096 && 0 <= part && part < nparts, GS_EINVAL,
                 "bad part %d of %d (at most 4096 parts)", part, nparts);
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        const int64_t nnz = g.nnz;
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * nnz, loc);
        if (nnz && g.symmetric) {
            jaccard_symmetric(c, dout, part, nparts);
        } else if (nnz) {  // directed: this part's edge range, zeros elsewhere
            const int64_t e0 = nnz * part / nparts, e1 = nnz * (part + 1) / nparts;
            GS_HIP(hipMemsetAsync(dout, 0, sizeof(double) * nnz, c->stream));
            if (e1 > e0) {
                hipEvent_t t0 = prof_begin(c);
                k_jaccard<<<grid_for(e1 - e0, 256), 256, 0, c->stream>>>(
                    g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.rows.as<int32_t>(),
                    g.tptr.as<int64_t>(), g.tidx.as<int32_t>(), e0, e1, dout + e0);
                GS_HIP(hipGetLastError());
                prof_end(c, t0, "jaccard", 0.0);
            }
        }
        finish_out(c, out, dout, sizeof(double) * nnz, loc);
    });
}

static void check_sharded_jaccard(gs_ctx *c, int nparts) {
    GS_CHECK(c, GS_EINVAL, "null context");
    GS_CHECK(nparts >= 1 && nparts <= 4096, GS_EINVAL, "bad part count %d", nparts);
    GS_CHECK(c->g.has_transpose, GS_ESTATE, "no graph set");
    GS_CHECK(c->g.symmetric, GS_EUNSUPPORTED,
             "owner-pair shares need a symmetric graph (use edge ranges on a directed one)");
}

int gs_jaccard_shares(gs_ctx *c, int nparts, int64_t *row_cut, int64_t *owner_off) {
    return guard([&] {
        check_sharded_jaccard(c, nparts);
        GS_HIP(hipSetDevice(c->device));
        const JacShares &sh = jaccard_shares(c, nparts);
        for (int r = 0; r <= nparts; ++r) {
            if (row_cut) row_cut[r] = sh.R(r);
            if (owner_off) owner_off[r] = sh.O(r);
        }
    });
}

int gs_jaccard_part_counts(gs_ctx *c, int part, int nparts, uint32_t *counts, int loc) {
    return guard([&] {
        check_sharded_jaccard(c, nparts);
        GS_CHECK(0 <= part && part < nparts, GS_EINVAL, "bad part %d of %d", part, nparts);
        GS_HIP(hipSetDevice(c->device));
        const JacShares &sh = jaccard_shares(c, nparts);
        const int64_t cnt = sh.O(part + 1) - sh.O(part);
        auto *d = (uint32_t *)out_device(c, c->outbuf, counts, sizeof(uint32_t) * cnt, loc);
        if (cnt) jaccard_symmetric(c, nullptr, part, nparts, 0, d);
        finish_out(c, counts, d, sizeof(uint32_t) * cnt, loc);
    });
}

int gs_jaccard_from_counts(gs_ctx *c, int nparts, const uint32_t *counts, int64_t stride,
                           int c_loc, double *out, int loc) {
    return guard([&] {
        check_sharded_jaccard(c, nparts);
        GS_CHECK(stride >= 0, GS_EINVAL, "negative stride");
        GS_HIP(hipSetDevice(c->device));
        const int64_t nnz = c->g.nnz;
        const uint32_t *dc = (const uint32_t *)to_device(c, c->inbuf, counts,
                                                         sizeof(uint32_t) * stride * nparts, c_loc);
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * nnz, loc);
        jaccard_from_counts(c, nparts, dc, stride, dout);
        finish_out(c, out, dout, sizeof(double) * nnz, loc);
    });
}

int gs_adamic_adar(gs_ctx *c, const double *cw, int c_loc, int64_t e0, int64_t e1, double *out,
                   int loc) {
    return guard([&] {
        check_range(c, e0, e1);
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        int64_t cnt = e1 - e0;
        const double *dc = (const double *)to_device(c, c->inbuf, cw, sizeof(double) * g.n, c_loc);
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * cnt, loc);
        if (cnt) {
            hipEvent_t t0 = prof_begin(c);
            k_adamic_adar<<<grid_for(cnt, 256), 256, 0, c->stream>>>(
                g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.rows.as<int32_t>(), dc, e0, e1,
                dout);
            GS_HIP(hipGetLastError());
            prof_end(c, t0, "adamic_adar", 0.0);
        }
        finish_out(c, out, dout, sizeof(double) * cnt, loc);
    });
}

int gs_degree(gs_ctx *c, int64_t e0, int64_t e1, double *out, int loc) {
    return guard([&] {
        check_range(c, e0, e1);
        GS_HIP(hipSetDevice(c->device));
        Graph &g = c->g;
        int64_t cnt = e1 - e0;
        double *deg = (double *)c->scratch[0].ensure(sizeof(double) * (g.n ? g.n : 1));
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * cnt, loc);
        if (g.n)
            k_row_sums<<<grid_for(g.n, 256), 256, 0, c->stream>>>(g.indptr.as<int64_t>(),
                                                                 g.data.as<double>(), g.n, deg);
        if (cnt)
            k_degree<<<grid_for(cnt, 256), 256, 0, c->stream>>>(g.rows.as<int32_t>(),
                                                               g.indices.as<int32_t>(), deg, e0,
                                                               e1, dout);
        GS_HIP(hipGetLastError());
        finish_out(c, out, dout, sizeof(double) * cnt, loc);
    });
}

int gs_feature_cosine_f32(gs_ctx *c, const float *x, int64_t f, int x_loc, int64_t e0, int64_t e1,
                          double *out, int loc) {
    return guard([&] { feature_cosine<float>(c, x, f, x_loc, e0, e1, out, loc); });
}

int gs_feature_cosine_f64(gs_ctx *c, const double *x, int64_t f, int x_loc, int64_t e0,
                          int64_t e1, double *out, int loc) {
    return guard([&] { feature_cosine<double>(c, x, f, x_loc, e0, e1, out, loc); });
}

}  // extern "C"
