// gs_exact_er.hip -- exact effective resistance (calculate_effective_resistance_scores,
// metrics.py:124-175) on the device, fp64 MFMA.
//
// The reference takes the dense pseudo-inverse of L + 1e-10 I by SVD and reads
// R(u,v) = P_uu + P_vv - 2 P_uv.  For u, v in one connected component C every
// component-constant term cancels in that form, so it equals the same form on
// M^{-1} with M = L + sum_C J_C / |C| (J_C = 1_C 1_C^T): M is SPD with the
// null vectors of L lifted to eigenvalue 1, and its condition number is that
// of L on the complement (no 1e10 direction).  The reference's own value
// carries the rounding of its 1e10/|C| component (1e-6 .. 5e-5 absolute on the
// fixtures); this computation is within ~1e-12 of an exact one.
//
// M^{-1} by Newton-Schulz, X <- 2X - X (M X), X0 = I / ||M||_inf (Gershgorin, so
// every eigenvalue of X0 M is in (0, 1]): two n^3 fp64 GEMMs per step on
// v_mfma_f64_16x16x4_f64, residual max|I - M X| checked every step.
#include "gs_internal.hpp"

namespace gs {

static constexpr int kGemmTile = 64;  // 64x64 output tile per 256-thread workgroup
static constexpr int kGemmK = 16;     // K slice staged in LDS

// C = alpha * A * B + beta * Cin  (N x N row-major, N a multiple of 64, fp64)
__global__ void __launch_bounds__(256) k_dgemm(int64_t N, const double *__restrict__ A,
                                               const double *__restrict__ B, double alpha,
                                               double beta, const double *__restrict__ Cin,
                                               double *__restrict__ C) {
    __shared__ double As[kGemmTile][kGemmK + 1];
    __shared__ double Bs[kGemmK][kGemmTile + 1];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t r0 = (int64_t)blockIdx.y * kGemmTile, c0 = (int64_t)blockIdx.x * kGemmTile;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;  // the wave's 32x32 quadrant
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    for (int64_t k0 = 0; k0 < N; k0 += kGemmK) {
        // stage A[r0..+64][k0..+16] and B[k0..+16][c0..+64]: 4 doubles per thread each
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + q * 256;
            const int ar = e / kGemmK, ac = e % kGemmK;
            As[ar][ac] = A[(r0 + ar) * N + k0 + ac];
            const int br = e / kGemmTile, bc = e % kGemmTile;
            Bs[br][bc] = B[(k0 + br) * N + c0 + bc];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kGemmK / 4; ++s) {
            const int kk = s * 4 + (lane >> 4);
            double a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = As[wr + i * 16 + (lane & 15)][kk];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Bs[kk][wc + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // C/D map of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = r0 + wr + i * 16 + (lane >> 4) + 4 * r;
                const int64_t col = c0 + wc + j * 16 + (lane & 15);
                const int64_t o = row * N + col;
                const double v = alpha * acc[i][j][r];
                C[o] = beta != 0.0 ? v + beta * Cin[o] : v;
            }
}

// value symmetry: A_uv == A_vu for every entry (the pattern check is ensure_transpose's)
__global__ void k_er_valsym(const int64_t *__restrict__ tpos, const double *__restrict__ d,
                            int64_t nnz, int *__restrict__ asym) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x)
        if (d[e] != d[tpos[e]]) atomicOr(asym, 1);
}

// connected components: min-label propagation with pointer jumping
__global__ void k_cc_init(int64_t n, int32_t *__restrict__ lab) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x)
        lab[u] = (int32_t)u;
}

__global__ void k_cc_hook(const int32_t *__restrict__ rows, const int32_t *__restrict__ ix,
                          int64_t nnz, int32_t *__restrict__ lab, int *__restrict__ changed) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t a = lab[rows[e]], b = lab[ix[e]];
        if (a < b) {
            atomicMin(&lab[b], a);
            *changed = 1;
        } else if (b < a) {
            atomicMin(&lab[a], b);
            *changed = 1;
        }
    }
}

__global__ void k_cc_jump(int64_t n, int32_t *__restrict__ lab) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        int32_t l = lab[u];
        while (lab[l] != l) l = lab[l];
        lab[u] = l;
    }
}

__global__ void k_cc_size(int64_t n, const int32_t *__restrict__ lab, int32_t *__restrict__ size) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x)
        atomicAdd(&size[lab[u]], 1);
}

// M = J-lift (1/|C| within a component), identity on the padding
__global__ void k_er_mfill(int64_t n, int64_t N, const int32_t *__restrict__ lab,
                           const int32_t *__restrict__ size, double *__restrict__ M) {
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < N * N;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = idx / N, j = idx % N;
        double v = 0.0;
        if (i < n && j < n) {
            if (lab[i] == lab[j]) v = 1.0 / (double)size[lab[i]];
        } else if (i == j) {
            v = 1.0;
        }
        M[idx] = v;
    }
}

// + L = D - A (degree = row sum of the multiplicities, metrics.py:159-163)
__global__ void k_er_laplace(int64_t n, int64_t N, const int64_t *__restrict__ ip,
                             const int32_t *__restrict__ ix, const double *__restrict__ d,
                             double *__restrict__ M) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        double deg = 0.0;
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) deg += d[e];
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) M[u * N + ix[e]] -= d[e];
        M[u * N + u] += deg;
    }
}

// Gershgorin bound max_i sum_j |M_ij| (one workgroup per row, max via bits)
__global__ void k_er_rownorm(int64_t N, const double *__restrict__ M,
                             unsigned long long *__restrict__ mx) {
    __shared__ double part[256];
    const int64_t i = blockIdx.x;
    double s = 0.0;
    for (int64_t j = threadIdx.x; j < N; j += blockDim.x) s += fabs(M[i * N + j]);
    part[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) atomicMax(mx, (unsigned long long)__double_as_longlong(part[0]));
}

__global__ void k_er_xinit(int64_t N, const unsigned long long *__restrict__ mx,
                           double *__restrict__ X) {
    const double c = 1.0 / __longlong_as_double((long long)*mx);
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < N * N;
         idx += (int64_t)gridDim.x * blockDim.x)
        X[idx] = (idx / N == idx % N) ? c : 0.0;
}

// max |I - T| (non-negative doubles order as their bits)
__global__ void k_er_resid(int64_t N, const double *__restrict__ T,
                           unsigned long long *__restrict__ mx) {
    double m = 0.0;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < N * N;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const double r = fabs((idx / N == idx % N ? 1.0 : 0.0) - T[idx]);
        m = r > m ? r : m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_down(m, o, 64);
        m = t > m ? t : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(mx, (unsigned long long)__double_as_longlong(m));
}

// r_eff in CSR order: (P_uu + P_vv) - 2 P_uv, then max(., 1e-10) (metrics.py:171-173)
__global__ void k_er_exact_scores(int64_t N, const int32_t *__restrict__ rows,
                                  const int32_t *__restrict__ ix, int64_t nnz,
                                  const double *__restrict__ X, double *__restrict__ out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = rows[e], v = ix[e];
        const double s = X[u * N + u] + X[v * N + v];
        const double t = 2.0 * X[u * N + v];
        const double r = s - t;
        out[e] = r > 1e-10 ? r : 1e-10;
    }
}

}  // namespace gs

using namespace gs;

extern "C" int gs_exact_er(gs_ctx *c, double *out, int loc, int32_t *iterations) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        Graph &g = c->g;
        ensure_transpose(c);
        GS_CHECK(g.symmetric, GS_EUNSUPPORTED,
                 "exact effective resistance needs a symmetric adjacency (metrics.py:138)");
        GS_CHECK(g.n <= 32768, GS_EUNSUPPORTED, "exact effective resistance is dense O(n^3): n=%lld",
                 (long long)g.n);
        GS_HIP(hipSetDevice(c->device));
        hipStream_t st = c->stream;
        const int64_t n = g.n, nnz = g.nnz;
        const int64_t N = ((n + kGemmTile - 1) / kGemmTile) * kGemmTile;
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * (nnz ? nnz : 1), loc);
        int32_t it_done = 0;
        if (n > 0) {
            auto *flags = (int *)c->buf("xer_flags").ensure(64);
            if (nnz) {
                GS_HIP(hipMemsetAsync(flags, 0, 4, st));
                k_er_valsym<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(g.tpos.as<int64_t>(),
                                                                     g.data.as<double>(), nnz, flags);
                int asym = 0;
                GS_HIP(hipMemcpyAsync(&asym, flags, 4, hipMemcpyDeviceToHost, st));
                GS_HIP(hipStreamSynchronize(st));
                GS_CHECK(!asym, GS_EUNSUPPORTED,
                         "exact effective resistance needs symmetric edge weights");
            }
            auto *lab = (int32_t *)c->buf("xer_lab").ensure(4 * n);
            auto *size = (int32_t *)c->buf("xer_size").ensure(4 * n);
            k_cc_init<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, lab);
            for (int round = 0; round < 4096; ++round) {
                GS_HIP(hipMemsetAsync(flags, 0, 4, st));
                if (nnz)
                    k_cc_hook<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(
                        g.rows.as<int32_t>(), g.indices.as<int32_t>(), nnz, lab, flags);
                k_cc_jump<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, lab);
                int ch = 0;
                GS_HIP(hipMemcpyAsync(&ch, flags, 4, hipMemcpyDeviceToHost, st));
                GS_HIP(hipStreamSynchronize(st));
                if (!ch) break;
            }
            GS_HIP(hipMemsetAsync(size, 0, 4 * n, st));
            k_cc_size<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, lab, size);
            const size_t mb = sizeof(double) * (size_t)N * (size_t)N;
            double *M = (double *)c->buf("xer_M").ensure(mb);
            double *X = (double *)c->buf("xer_X").ensure(mb);
            double *X2 = (double *)c->buf("xer_X2").ensure(mb);
            double *T = (double *)c->buf("xer_T").ensure(mb);
            auto *mx = (unsigned long long *)c->buf("xer_mx").ensure(64);
            k_er_mfill<<<grid_for(N * N, 256, 65536), 256, 0, st>>>(n, N, lab, size, M);
            k_er_laplace<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, N, g.indptr.as<int64_t>(),
                                                                g.indices.as<int32_t>(),
                                                                g.data.as<double>(), M);
            GS_HIP(hipMemsetAsync(mx, 0, 64, st));
            k_er_rownorm<<<(unsigned)N, 256, 0, st>>>(N, M, mx);
            k_er_xinit<<<grid_for(N * N, 256, 65536), 256, 0, st>>>(N, mx, X);
            const dim3 gg((unsigned)(N / kGemmTile), (unsigned)(N / kGemmTile));
            const double flops = 2.0 * (double)N * (double)N * (double)N;
            double prev = 1e300;
            for (int it = 0; it < 256; ++it) {
                hipEvent_t t0 = prof_begin(c);
                k_dgemm<<<gg, 256, 0, st>>>(N, M, X, 1.0, 0.0, nullptr, T);  // T = M X
                prof_end(c, t0, "exact_er_dgemm", flops);
                GS_HIP(hipMemsetAsync(mx + 1, 0, 8, st));
                k_er_resid<<<grid_for(N * N, 256, 16384), 256, 0, st>>>(N, T, mx + 1);
                unsigned long long rb = 0;
                GS_HIP(hipMemcpyAsync(&rb, mx + 1, 8, hipMemcpyDeviceToHost, st));
                GS_HIP(hipStreamSynchronize(st));
                double res;
                memcpy(&res, &rb, 8);
                it_done = it;
                // converged, or rounding has taken over: in the quadratic phase each
                // step squares the residual, at the rounding floor it stalls
                if (res < 1e-13 || (prev < 1e-3 && res > 0.5 * prev)) break;
                prev = res;
                t0 = prof_begin(c);
                k_dgemm<<<gg, 256, 0, st>>>(N, X, T, -1.0, 2.0, X, X2);  // X2 = 2X - X T
                prof_end(c, t0, "exact_er_dgemm", flops);
                std::swap(X, X2);
                GS_CHECK(it < 255, GS_EHIP, "Newton-Schulz did not converge (residual %g)", res);
            }
            if (nnz)
                k_er_exact_scores<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(
                    N, g.rows.as<int32_t>(), g.indices.as<int32_t>(), nnz, X, dout);
            GS_HIP(hipGetLastError());
        }
        finish_out(c, out, dout, sizeof(double) * nnz, loc);
        if (iterations) *iterations = it_done;
    });
}
