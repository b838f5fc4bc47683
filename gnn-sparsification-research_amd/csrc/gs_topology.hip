// gs_topology.hip -- compute_topology_metrics (metrics.py:445-520) on the
// device: common-neighbour counts, the average clustering coefficient in
// NetworkX's exact operation order, connected components, and the algebraic
// connectivity (Fiedler value) of a connected graph.
//
// Clustering (nx.average_clustering): per node t(v) = sum over its entries of
// |N(u) ∩ N(v)| (the owner-side Jaccard intersection kernels in count mode),
// c_v = 0 if t == 0 else t / (d (d - 1)) (one correctly rounded division of
// exact integers, as Python's int / int), summed left to right from 0 in node
// order (Python's sum over the dict) and divided by n.  The caller passes the
// self-loop-free symmetric pattern (NetworkX drops v from its own neighbour set).
//
// Fiedler value: lambda_2(L) = 1 / lambda_max(L^+), L^+ = P G P with G the
// grounded inverse (zero at the ground node) and P = I - 11^T / n; G x =
// W^T (W x) with W = L_M^{-1} from gs_exact_er.hip's blocked Cholesky of the
// grounded M.  lambda_max(P G P) by Lanczos with full (classical Gram-Schmidt,
// twice) reorthogonalisation; the tridiagonal's largest eigenvalue by
// Sturm-count bisection, all on the device.
#include <cmath>

#include "gs_internal.hpp"

namespace gs {

// c_v per node from the per-entry counts (CSR order)
__global__ void k_clust_node(const int64_t *__restrict__ ip, const double *__restrict__ cnt,
                             int64_t n, double *__restrict__ cv) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x) {
        double t = 0.0;  // exact: integer counts far below 2^53
        for (int64_t e = ip[v]; e < ip[v + 1]; ++e) t += cnt[e];
        const double d = (double)(ip[v + 1] - ip[v]);
        cv[v] = t == 0.0 ? 0.0 : t / (d * (d - 1.0));
    }
}

// Python's sum(values) / len: a left fold from 0 in node order (one thread)
__global__ void k_fold_mean(const double *__restrict__ cv, int64_t n, double *__restrict__ out) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    double s = 0.0;
    for (int64_t v = 0; v < n; ++v) s = s + cv[v];
    out[0] = n ? s / (double)n : 0.0;
}

__global__ void k_comp_sizes(const int32_t *__restrict__ lab, int64_t n,
                             unsigned long long *__restrict__ size) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&size[lab[v]], 1ull);
}

__global__ void k_comp_stats(const int32_t *__restrict__ lab,
                             const unsigned long long *__restrict__ size, int64_t n,
                             unsigned long long *__restrict__ stats) {
    for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < n;
         v += (int64_t)gridDim.x * blockDim.x)
        if (lab[v] == v) {
            atomicAdd(&stats[0], 1ull);
            atomicMax(&stats[1], size[v]);
        }
}

// ---------------------------------------------------------------- Fiedler
static constexpr int kLzThreads = 1024;
static constexpr int kLzWaves = kLzThreads / 64;

// y_i = sum_{k <= i} W_ik x_k (W lower triangular), x zero at flagged nodes
__global__ void __launch_bounds__(256) k_gemv_lower(int64_t N, const double *__restrict__ W,
                                                    const double *__restrict__ x,
                                                    const uint8_t *__restrict__ flag,
                                                    double *__restrict__ y) {
    const int64_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= N) return;
    double s = 0.0;
    for (int64_t k = lane; k <= i; k += 64) s += flag[k] ? 0.0 : W[i * N + k] * x[k];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) y[i] = s;
}

// z_k = sum_{i >= k} U_ki y_i (U = W^T upper triangular), zero at flagged nodes
__global__ void __launch_bounds__(256) k_gemv_upper(int64_t N, const double *__restrict__ U,
                                                    const double *__restrict__ y,
                                                    const uint8_t *__restrict__ flag,
                                                    double *__restrict__ z) {
    const int64_t k = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (k >= N) return;
    double s = 0.0;
    for (int64_t i = k + lane; i < N; i += 64) s += U[k * N + i] * y[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) z[k] = flag[k] ? 0.0 : s;
}

__device__ double lz_block_sum(double v, double *red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < kLzWaves; ++w) s += red[w];
    return s;
}

// x = P v_j (mean over the n real nodes removed), the input of G
__global__ void __launch_bounds__(kLzThreads) k_lz_in(int64_t n, const double *__restrict__ v,
                                                      double *__restrict__ x) {
    __shared__ double red[kLzWaves];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kLzThreads) s += v[i];
    const double mean = lz_block_sum(s, red) / (double)n;
    for (int64_t i = threadIdx.x; i < n; i += kLzThreads) x[i] = v[i] - mean;
}

// v_0: a fixed pseudo-random vector (mean removed, unit norm), deterministic
__global__ void __launch_bounds__(kLzThreads) k_lz_init(int64_t n, double *__restrict__ v) {
    __shared__ double red[kLzWaves];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kLzThreads) {
        const uint64_t h = ((uint64_t)i + 1) * 0x9E3779B97F4A7C15ull;
        v[i] = (double)(h >> 11) * 0x1p-53 - 0.5;
        s += v[i];
    }
    const double mean = lz_block_sum(s, red) / (double)n;
    s = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += kLzThreads) {
        v[i] -= mean;
        s += v[i] * v[i];
    }
    const double nrm = sqrt(lz_block_sum(s, red));
    for (int64_t i = threadIdx.x; i < n; i += kLzThreads) v[i] /= nrm;
}

// Sturm count: eigenvalues of the (m x m) tridiagonal (a, b) below x
__device__ int lz_sturm(const double *a, const double *b, int m, double x) {
    int cnt = 0;
    double q = 1.0;
    for (int i = 0; i < m; ++i) {
        const double bb = i ? b[i - 1] * b[i - 1] : 0.0;
        q = a[i] - x - (i ? bb / q : 0.0);
        if (q == 0.0) q = 1e-300;
        if (q < 0.0) ++cnt;
    }
    return cnt;
}

// One Lanczos step on w = G x (the output of the two GEMVs): w <- P w,
// alpha_j, three-term recurrence, CGS2 against v_0..v_j, beta_j, v_{j+1};
// theta = largest eigenvalue of T_{j+1} by bisection (every step: m <= 400).
__global__ void __launch_bounds__(kLzThreads) k_lz_step(int64_t n, int64_t ldv, int j,
                                                        double *__restrict__ V,
                                                        double *__restrict__ w,
                                                        double *__restrict__ al,
                                                        double *__restrict__ be,
                                                        double *__restrict__ c,
                                                        double *__restrict__ theta) {
    __shared__ double red[kLzWaves];
    __shared__ double s_c[512];
    const int tid = threadIdx.x;
    // P w
    double s = 0.0;
    for (int64_t i = tid; i < n; i += kLzThreads) s += w[i];
    const double mean = lz_block_sum(s, red) / (double)n;
    for (int64_t i = tid; i < n; i += kLzThreads) w[i] -= mean;
    __syncthreads();
    const double *vj = V + (int64_t)j * ldv;
    s = 0.0;
    for (int64_t i = tid; i < n; i += kLzThreads) s += vj[i] * w[i];
    const double a = lz_block_sum(s, red);
    const double bprev = j ? be[j - 1] : 0.0;
    const double *vp = j ? V + (int64_t)(j - 1) * ldv : vj;
    for (int64_t i = tid; i < n; i += kLzThreads) w[i] = w[i] - a * vj[i] - bprev * vp[i];
    __syncthreads();
    // classical Gram-Schmidt, twice: one wave per basis vector's dot
    for (int pass = 0; pass < 2; ++pass) {
        const int wv = tid >> 6, lane = tid & 63;
        for (int q = wv; q <= j; q += kLzWaves) {
            const double *vq = V + (int64_t)q * ldv;
            double d = 0.0;
            for (int64_t i = lane; i < n; i += 64) d += vq[i] * w[i];
            for (int o = 32; o > 0; o >>= 1) d += __shfl_down(d, o, 64);
            if (lane == 0) s_c[q] = d;
        }
        __syncthreads();
        for (int64_t i = tid; i < n; i += kLzThreads) {
            double t = w[i];
            for (int q = 0; q <= j; ++q) t -= s_c[q] * V[(int64_t)q * ldv + i];
            w[i] = t;
        }
        __syncthreads();
    }
    s = 0.0;
    for (int64_t i = tid; i < n; i += kLzThreads) s += w[i] * w[i];
    const double b = sqrt(lz_block_sum(s, red));
    double *vn = V + (int64_t)(j + 1) * ldv;
    for (int64_t i = tid; i < n; i += kLzThreads) vn[i] = b > 0.0 ? w[i] / b : 0.0;
    if (tid == 0) {
        al[j] = a;
        be[j] = b;
        // largest eigenvalue of T (j+1 x j+1): Gershgorin bracket, bisection
        const int m = j + 1;
        double lo = 1e300, hi = -1e300;
        for (int i = 0; i < m; ++i) {
            const double r = (i ? fabs(be[i - 1]) : 0.0) + (i + 1 < m ? fabs(be[i]) : 0.0);
            lo = fmin(lo, al[i] - r);
            hi = fmax(hi, al[i] + r);
        }
        for (int it = 0; it < 200 && hi - lo > 1e-15 * fabs(hi); ++it) {
            const double mid = 0.5 * (lo + hi);
            if (lz_sturm(al, be, m, mid) < m) lo = mid;  // some eigenvalue above mid
            else hi = mid;
        }
        theta[j] = hi;
        c[0] = b;
    }
}

}  // namespace gs

using namespace gs;

extern "C" {

int gs_common_neighbors(gs_ctx *c, double *out, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        Graph &g = c->g;
        ensure_transpose(c);
        GS_CHECK(g.symmetric, GS_EUNSUPPORTED, "common-neighbour counts need a symmetric graph");
        GS_HIP(hipSetDevice(c->device));
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * (g.nnz ? g.nnz : 1), loc);
        if (g.nnz) jaccard_symmetric(c, dout, 0, 1, 1);
        finish_out(c, out, dout, sizeof(double) * g.nnz, loc);
    });
}

int gs_clustering(gs_ctx *c, double *avg, double *per_node, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        Graph &g = c->g;
        ensure_transpose(c);
        GS_CHECK(g.symmetric, GS_EUNSUPPORTED, "clustering needs a symmetric graph");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        const int64_t n = g.n, nnz = g.nnz;
        double *cnt = (double *)c->buf("topo_cnt").ensure(sizeof(double) * (nnz ? nnz : 1));
        double *cv = per_node && loc == GS_DEVICE
                         ? per_node
                         : (double *)c->buf("topo_cv").ensure(sizeof(double) * (n ? n : 1));
        double *dav = (double *)c->buf("topo_avg").ensure(sizeof(double));
        if (nnz) jaccard_symmetric(c, cnt, 0, 1, 1);
        if (n) {
            if (nnz)
                k_clust_node<<<grid_for(n, 256, 8192), 256, 0, st>>>(g.indptr.as<int64_t>(), cnt, n,
                                                                     cv);
            else
                GS_HIP(hipMemsetAsync(cv, 0, sizeof(double) * n, st));
        }
        k_fold_mean<<<1, 64, 0, st>>>(cv, n, dav);
        GS_HIP(hipGetLastError());
        GS_HIP(hipMemcpyAsync(avg, dav, sizeof(double), hipMemcpyDeviceToHost, st));
        if (per_node && loc != GS_DEVICE && n)
            GS_HIP(hipMemcpyAsync(per_node, cv, sizeof(double) * n, hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));
    });
}

int gs_components(gs_ctx *c, int32_t *labels, int loc, int64_t *count, int64_t *largest) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        Graph &g = c->g;
        GS_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        const int64_t n = g.n;
        int32_t *lab = components(c);
        auto *size = (unsigned long long *)c->buf("topo_size").ensure(8 * (n ? n : 1));
        auto *stats = (unsigned long long *)c->buf("topo_stats").ensure(16);
        GS_HIP(hipMemsetAsync(stats, 0, 16, st));
        if (n) {
            GS_HIP(hipMemsetAsync(size, 0, 8 * n, st));
            k_comp_sizes<<<grid_for(n, 256, 8192), 256, 0, st>>>(lab, n, size);
            k_comp_stats<<<grid_for(n, 256, 8192), 256, 0, st>>>(lab, size, n, stats);
        }
        unsigned long long h[2] = {0, 0};
        GS_HIP(hipMemcpyAsync(h, stats, 16, hipMemcpyDeviceToHost, st));
        if (labels && n)
            GS_HIP(hipMemcpyAsync(labels, lab, 4 * n,
                                  loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                  st));
        GS_HIP(hipStreamSynchronize(st));
        if (count) *count = (int64_t)h[0];
        if (largest) *largest = (int64_t)h[1];
    });
}

int gs_fiedler(gs_ctx *c, double tol, int32_t max_iter, double *value, int32_t *iterations) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        Graph &g = c->g;
        ensure_transpose(c);
        GS_CHECK(g.symmetric, GS_EUNSUPPORTED, "algebraic connectivity needs a symmetric graph");
        const int64_t n = g.n;
        GS_CHECK(n >= 2, GS_EINVAL, "algebraic connectivity needs n >= 2");
        GS_CHECK(n <= 32768, GS_EUNSUPPORTED, "algebraic connectivity here is dense O(n^3): n=%lld",
                 (long long)n);
        GS_CHECK(max_iter >= 2 && max_iter <= 500, GS_EINVAL, "max_iter in [2, 500]");
        GS_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        int64_t ncomp = 0;
        {
            int32_t *lab = components(c);
            auto *stats = (unsigned long long *)c->buf("topo_stats").ensure(16);
            auto *size = (unsigned long long *)c->buf("topo_size").ensure(8 * n);
            GS_HIP(hipMemsetAsync(stats, 0, 16, st));
            GS_HIP(hipMemsetAsync(size, 0, 8 * n, st));
            k_comp_sizes<<<grid_for(n, 256, 8192), 256, 0, st>>>(lab, n, size);
            k_comp_stats<<<grid_for(n, 256, 8192), 256, 0, st>>>(lab, size, n, stats);
            unsigned long long h[2];
            GS_HIP(hipMemcpyAsync(h, stats, 16, hipMemcpyDeviceToHost, st));
            GS_HIP(hipStreamSynchronize(st));
            ncomp = (int64_t)h[0];
        }
        GS_CHECK(ncomp == 1, GS_EINVAL, "algebraic connectivity: graph has %lld components",
                 (long long)ncomp);
        // ground node 0 (any node grounds a connected graph); padding rows identity
        const int64_t N = ((n + 63) / 64) * 64;
        auto *flag = (uint8_t *)c->buf("topo_flag").ensure(N);
        GS_HIP(hipMemsetAsync(flag, 0, N, st));
        GS_HIP(hipMemsetAsync(flag, 1, 1, st));
        if (N > n) GS_HIP(hipMemsetAsync(flag + n, 1, N - n, st));
        const size_t mb = sizeof(double) * (size_t)N * (size_t)N;
        double *A = (double *)c->buf("xer_X").ensure(mb);
        double *W = (double *)c->buf("xer_S").ensure(mb);
        grounded_inverse(c, N, flag, A, W);
        transpose_square(c, N, W, A);  // A = U = W^T: G x = U (W x)
        const int64_t ldv = (n + 63) & ~(int64_t)63;
        double *V = (double *)c->buf("lz_V").ensure(sizeof(double) * (size_t)(max_iter + 1) * ldv);
        double *x = (double *)c->buf("lz_x").ensure(sizeof(double) * N);
        double *y = (double *)c->buf("lz_y").ensure(sizeof(double) * N);
        double *w = (double *)c->buf("lz_w").ensure(sizeof(double) * N);
        double *ab = (double *)c->buf("lz_ab").ensure(sizeof(double) * (3 * (size_t)max_iter + 8));
        double *al = ab, *be = ab + max_iter, *th = ab + 2 * max_iter, *cb = ab + 3 * max_iter;
        k_lz_init<<<1, kLzThreads, 0, st>>>(n, V);
        double prev = 0.0, theta = 0.0;
        int32_t done = 0;
        for (int j = 0; j < max_iter; ++j) {
            k_lz_in<<<1, kLzThreads, 0, st>>>(n, V + (int64_t)j * ldv, x);
            k_gemv_lower<<<(unsigned)((N + 3) / 4), 256, 0, st>>>(N, W, x, flag, y);
            k_gemv_upper<<<(unsigned)((N + 3) / 4), 256, 0, st>>>(N, A, y, flag, w);
            k_lz_step<<<1, kLzThreads, 0, st>>>(n, ldv, j, V, w, al, be, cb, th);
            GS_HIP(hipGetLastError());
            done = j + 1;
            if (j % 4 != 3 && j + 1 < max_iter && j + 1 < n - 1) continue;
            double h[2];
            GS_HIP(hipMemcpyAsync(&h[0], th + j, sizeof(double), hipMemcpyDeviceToHost, st));
            GS_HIP(hipMemcpyAsync(&h[1], be + j, sizeof(double), hipMemcpyDeviceToHost, st));
            GS_HIP(hipStreamSynchronize(st));
            theta = h[0];
            // converged, an invariant subspace (beta ~ 0), or the Krylov space is full
            if (fabs(theta - prev) <= tol * fabs(theta) || !(h[1] > 1e-14 * fabs(theta)) ||
                j + 1 >= n - 1)
                break;
            prev = theta;
        }
        GS_CHECK(theta > 0.0, GS_EHIP, "Lanczos: non-positive lambda_max(L^+)");
        if (value) *value = 1.0 / theta;
        if (iterations) *iterations = done;
    });
}

}  // extern "C"
