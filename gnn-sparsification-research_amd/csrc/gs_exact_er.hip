// gs_exact_er.hip -- exact effective resistance (calculate_effective_resistance_scores,
// metrics.py:124-175) on the device, fp64 MFMA.
//
// The reference takes the dense pseudo-inverse of L + 1e-10 I by SVD and reads
// R(u,v) = P_uu + P_vv - 2 P_uv.  Within a connected component that is the
// effective resistance, which grounding one node g per component computes
// exactly: with M = L with row/column g replaced by the identity (SPD, sparse)
// and G = M^{-1} with row/column g zeroed, R(u,v) = G_uu + G_vv - 2 G_uv.  The
// reference's own value carries the rounding of its 1e10/|C| direction (1e-6 ..
// 5e-5 absolute on the fixtures); this computation has none of it.  g = the
// component's node of largest degree (smallest id on ties).
//
// M^{-1} by Newton-Schulz in its symmetric form, X <- 2X - X (M X) with
// X0 = I / ||M||_inf (Gershgorin, so every eigenvalue of X0 M is in (0, 1]):
// S = M X is a sparse-times-dense product (nnz N per step, HBM-bound), X S =
// X M X is exactly symmetric in exact arithmetic for any symmetric X, so only
// its upper-triangle tiles run (N^3 flops per step on v_mfma_f64_16x16x4_f64)
// and X stays exactly symmetric.  ||I - M X||_F is folded into the S kernel.
#include <cmath>
#include <cstring>

#include "gs_internal.hpp"

namespace gs {

static constexpr int kGemmPad = 64;  // N is padded to a multiple of this
static constexpr int kGemmK = 16;    // K slice staged in LDS

// Workgroup -> output tile.  Dispatch deals consecutive workgroup ids round-robin
// over the 8 XCDs; regroup so each XCD walks a contiguous run of tiles (shared
// A rows / B columns stay in its own L2).  SYM: only tiles bi <= bj (row-major
// over the upper triangle), the result mirrored into (bj, bi).
template <bool SYM>
__device__ __forceinline__ void gemm_tile(int nb, int &bi, int &bj) {
    const int nblk = gridDim.x;
    int t = blockIdx.x;
    if ((nblk & 7) == 0) t = (t & 7) * (nblk >> 3) + (t >> 3);
    if (!SYM) {
        bi = t / nb;
        bj = t % nb;
        return;
    }
    // row bi starts at s(bi) = bi*nb - bi*(bi-1)/2
    const double q = 2.0 * nb + 1.0;
    int r = (int)((q - sqrt(q * q - 8.0 * t)) * 0.5);
    while (r > 0 && (int64_t)r * nb - (int64_t)r * (r - 1) / 2 > t) --r;
    while ((int64_t)(r + 1) * nb - (int64_t)(r + 1) * r / 2 <= t) ++r;
    bi = r;
    bj = r + (t - (r * nb - r * (r - 1) / 2));
}

// C = alpha * A * B + beta * Cin  (N x N row-major, N a multiple of TM, fp64).
// TM x TM output tile per 256-thread workgroup, four waves in 2x2, each wave
// (TM/2)^2 as (TM/32)^2 v_mfma_f64_16x16x4_f64 tiles.  K advances 16 at a time
// through LDS; the next slice is loaded into registers (16-byte loads) while
// the current one feeds the MFMAs.  SYM: the product is symmetric (X (M X) with
// X, M symmetric): upper-triangle tiles only, each written to both triangles.
template <bool SYM, int TM>
__global__ void __launch_bounds__(256) k_dgemm(int64_t N, const double *__restrict__ A,
                                               const double *__restrict__ B, double alpha,
                                               double beta, const double *__restrict__ Cin,
                                               double *__restrict__ C) {
    constexpr int FT = TM / 32;          // MFMA tiles per wave per dimension
    constexpr int LA = TM * kGemmK / 512;  // 16-byte loads per thread per operand
    __shared__ double As[TM][kGemmK + 2];
    __shared__ double Bs[kGemmK][TM + 2];
    typedef double d2 __attribute__((ext_vector_type(2)));
    typedef double d4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int bi, bj;
    gemm_tile<SYM>((int)(N / TM), bi, bj);
    const int64_t r0 = (int64_t)bi * TM, c0 = (int64_t)bj * TM;
    const int wr = (wave >> 1) * (TM / 2), wc = (wave & 1) * (TM / 2);
    d4 acc[FT][FT];
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    d2 ra[LA], rb[LA];
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int q = 0; q < LA; ++q) {
            const int e = tid + q * 256;  // d2 index within the slice
            const int ar = e / (kGemmK / 2), ac = (e % (kGemmK / 2)) * 2;
            ra[q] = *(const d2 *)(A + (r0 + ar) * N + k0 + ac);
            const int br = e / (TM / 2), bc = (e % (TM / 2)) * 2;
            rb[q] = *(const d2 *)(B + (k0 + br) * N + c0 + bc);
        }
    };
    auto stage = [&]() {
#pragma unroll
        for (int q = 0; q < LA; ++q) {
            const int e = tid + q * 256;
            const int ar = e / (kGemmK / 2), ac = (e % (kGemmK / 2)) * 2;
            *(d2 *)&As[ar][ac] = ra[q];
            const int br = e / (TM / 2), bc = (e % (TM / 2)) * 2;
            *(d2 *)&Bs[br][bc] = rb[q];
        }
    };
    load(0);
    for (int64_t k0 = 0; k0 < N; k0 += kGemmK) {
        stage();
        __syncthreads();
        if (k0 + kGemmK < N) load(k0 + kGemmK);
#pragma unroll
        for (int s = 0; s < kGemmK / 4; ++s) {
            const int kk = s * 4 + (lane >> 4);
            double a[FT], b[FT];
#pragma unroll
            for (int i = 0; i < FT; ++i) a[i] = As[wr + i * 16 + (lane & 15)][kk];
#pragma unroll
            for (int j = 0; j < FT; ++j) b[j] = Bs[kk][wc + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < FT; ++i)
#pragma unroll
                for (int j = 0; j < FT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    // C/D map of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int i = 0; i < FT; ++i)
#pragma unroll
        for (int j = 0; j < FT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t row = r0 + wr + i * 16 + (lane >> 4) + 4 * r;
                const int64_t col = c0 + wc + j * 16 + (lane & 15);
                const int64_t o = row * N + col;
                const double v = alpha * acc[i][j][r];
                const double w = beta != 0.0 ? v + beta * Cin[o] : v;
                C[o] = w;
                if (SYM && bi != bj) C[col * N + row] = w;
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

// grounded node per component: largest row length, smallest id on ties
__global__ void k_er_ground_pick(int64_t n, const int64_t *__restrict__ ip,
                                 const int32_t *__restrict__ lab,
                                 unsigned long long *__restrict__ best) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        const unsigned long long key = ((unsigned long long)(ip[u + 1] - ip[u]) << 32) |
                                       (unsigned long long)(0xffffffffu - (uint32_t)u);
        atomicMax(&best[lab[u]], key);
    }
}

// flag[u] = 1 for identity rows of M (grounded nodes and the padding up to N)
__global__ void k_er_ground_mark(int64_t n, int64_t N, const int32_t *__restrict__ lab,
                                 const unsigned long long *__restrict__ best,
                                 uint8_t *__restrict__ flag) {
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < N;
         u += (int64_t)gridDim.x * blockDim.x) {
        if (u >= n) {
            flag[u] = 1;
            continue;
        }
        const uint32_t g = 0xffffffffu - (uint32_t)(best[lab[u]] & 0xffffffffu);
        flag[u] = g == (uint32_t)u;
    }
}

// Gershgorin bound ||M||_inf (max via the bits of a non-negative double)
__global__ void k_er_rownorm(int64_t n, const int64_t *__restrict__ ip,
                             const int32_t *__restrict__ ix, const double *__restrict__ d,
                             const uint8_t *__restrict__ flag, unsigned long long *__restrict__ mx) {
    double m = 1.0;  // identity rows
    for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        if (flag[u]) continue;
        double deg = 0.0, diag = 0.0, off = 0.0;
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            deg += d[e];
            if (ix[e] == u) diag += d[e];
            else if (!flag[ix[e]]) off += d[e];
        }
        const double r = fabs(deg - diag) + off;
        m = r > m ? r : m;
    }
    for (int o = 32; o > 0; o >>= 1) {
        const double t = __shfl_down(m, o, 64);
        m = t > m ? t : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax(mx, (unsigned long long)__double_as_longlong(m));
}

__global__ void k_er_xinit(int64_t N, const unsigned long long *__restrict__ mx,
                           double *__restrict__ X) {
    const double c = 1.0 / __longlong_as_double((long long)*mx);
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < N * N;
         idx += (int64_t)gridDim.x * blockDim.x)
        X[idx] = (idx / N == idx % N) ? c : 0.0;
}

// S = M X, row i of S from row i of the CSR: (deg_i - A_ii) X_i - sum A_ij X_j over
// non-grounded j != i; S_i = X_i on identity rows.  One workgroup per (row,
// 256-column slice); each block also leaves its share of ||I - S||_F^2.
__global__ void __launch_bounds__(256) k_er_spmm(int64_t n, int64_t N, const int64_t *__restrict__ ip,
                                                 const int32_t *__restrict__ ix,
                                                 const double *__restrict__ d,
                                                 const uint8_t *__restrict__ flag,
                                                 const double *__restrict__ X,
                                                 double *__restrict__ S, double *__restrict__ part) {
    __shared__ double red[4];
    const int64_t slices = (N + 255) / 256;
    const int64_t i = blockIdx.x / slices;
    const int64_t j = (blockIdx.x % slices) * 256 + threadIdx.x;
    double v = 0.0;
    if (j >= N) {
        // past the last column: contributes nothing
    } else if (flag[i]) {
        v = X[i * N + j];
    } else {
        double deg = 0.0, diag = 0.0, acc = 0.0;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e) {
            const int32_t k = ix[e];
            const double w = d[e];
            deg += w;
            if (k == i) diag += w;
            else if (!flag[k]) acc += w * X[(int64_t)k * N + j];
        }
        v = (deg - diag) * X[i * N + j] - acc;
    }
    if (j < N) S[i * N + j] = v;
    const double r = j < N ? (i == j ? 1.0 : 0.0) - v : 0.0;
    double s2 = r * r;
    for (int o = 32; o > 0; o >>= 1) s2 += __shfl_down(s2, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s2;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ||I - S||_F from the per-block shares, folded in a fixed order (deterministic)
__global__ void __launch_bounds__(256) k_er_resid_fin(const double *__restrict__ part, int64_t np,
                                                      double *__restrict__ res) {
    __shared__ double red[256];
    double s = 0.0;
    for (int64_t i = threadIdx.x; i < np; i += 256) s += part[i];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *res = sqrt(red[0]);
}

// r_eff in CSR order: (G_uu + G_vv) - 2 G_uv, then max(., 1e-10) (metrics.py:171-173);
// G = X with grounded rows/columns read as zero
__global__ void k_er_exact_scores(int64_t N, const int32_t *__restrict__ rows,
                                  const int32_t *__restrict__ ix, int64_t nnz,
                                  const uint8_t *__restrict__ flag,
                                  const double *__restrict__ X, double *__restrict__ out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t u = rows[e], v = ix[e];
        const bool fu = flag[u], fv = flag[v];
        const double guu = fu ? 0.0 : X[u * N + u];
        const double gvv = fv ? 0.0 : X[v * N + v];
        const double guv = (fu || fv) ? 0.0 : X[u * N + v];
        const double r = (guu + gvv) - 2.0 * guv;
        out[e] = r > 1e-10 ? r : 1e-10;
    }
}

// ---------------------------------------------------------------- Cholesky path
// G = M^{-1} from a blocked Cholesky factorisation M = L L^T and W = L^{-1}
// (64 x 64 blocks; N^3/3 + N^3/3 flops instead of Newton-Schulz's ~N^3 per step
// over ~log2(cond M) steps), G_uv = (W^T W)_uv = sum_{k >= max(u,v)} W_ku W_kv
// read from U = W^T.  Per block step k:
//   k_chol_diag       : A_kk = L_kk L_kk^T in LDS, D_k = L_kk^{-1}
//   k_tile_mm<PANEL>  : A_ik <- A_ik D_k^T                 (i > k)
//   k_tile_mm<UPDATE> : A_ij -= A_ik A_jk^T                 (k < j <= i)
// then, with W = I:
//   k_tile_mm<INVROW> : W_kj <- D_k W_kj                    (j <= k)
//   k_tile_mm<INVUPD> : W_ij -= A_ik W_kj                   (i > k, j <= k)
// Every tile product is 64 x 64 x 64 on v_mfma_f64_16x16x4_f64 (four waves of
// 2 x 2 MFMA tiles), both operands staged whole in LDS.
static constexpr int kCb = 64;

__global__ void k_er_dense_rows(int64_t n, int64_t N, const int64_t *__restrict__ ip,
                                const int32_t *__restrict__ ix, const double *__restrict__ d,
                                const uint8_t *__restrict__ flag, double *__restrict__ A) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N;
         i += (int64_t)gridDim.x * blockDim.x) {
        if (i >= n || flag[i]) {
            A[i * N + i] = 1.0;
            continue;
        }
        double deg = 0.0, diag = 0.0;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e) {
            const int32_t k = ix[e];
            deg += d[e];
            if (k == i) diag += d[e];
            else if (!flag[k]) A[i * N + k] = -d[e];
        }
        A[i * N + i] = deg - diag;
    }
}

__global__ void k_er_identity(int64_t N, double *__restrict__ W) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < N;
         i += (int64_t)gridDim.x * blockDim.x)
        W[i * N + i] = 1.0;
}

// factor the diagonal block in LDS (right-looking, all 256 threads); *bad = 1 on
// a non-positive pivot.  D = L^{-1} by 2 x 2 blocks of 32:
// T11 = L11^{-1}, T22 = L22^{-1} (one thread per column, both halves at once),
// then T21 = -T22 (L21 T11) on all 256 threads.
__global__ void __launch_bounds__(256) k_chol_diag(int64_t N, int k, double *__restrict__ A,
                                                   double *__restrict__ D, int *__restrict__ bad) {
    __shared__ double S[kCb][kCb + 1];
    __shared__ double T[kCb][kCb + 1];
    __shared__ double Z[32][33];
    const int tid = threadIdx.x;
    double *Akk = A + (int64_t)k * kCb * N + (int64_t)k * kCb;
    for (int e = tid; e < kCb * kCb; e += 256) {
        const int r = e / kCb, c = e % kCb;
        S[r][c] = c <= r ? Akk[(int64_t)r * N + c] : 0.0;
        T[r][c] = 0.0;
    }
    __syncthreads();
    for (int j = 0; j < kCb; ++j) {
        if (tid == 0) {
            const double p = S[j][j];
            if (!(p > 0.0)) *bad = 1;
            S[j][j] = sqrt(p > 0.0 ? p : 1.0);
        }
        __syncthreads();
        for (int i = j + 1 + tid; i < kCb; i += 256) S[i][j] = S[i][j] / S[j][j];
        __syncthreads();
        const int m = kCb - 1 - j;
        for (int e = tid; e < m * m; e += 256) {
            const int i = j + 1 + e / m, l = j + 1 + e % m;
            if (l <= i) S[i][l] -= S[i][j] * S[l][j];
        }
        __syncthreads();
    }
    // diagonal halves: thread c < 32 -> column c of T11, 32 <= c < 64 -> column of T22
    if (tid < 64) {
        const int c = tid, lo = c < 32 ? 0 : 32, hi = lo + 32;
        for (int i = c; i < hi; ++i) {
            double s = i == c ? 1.0 : 0.0;
            for (int q = c; q < i; ++q) s -= S[i][q] * T[q][c];
            T[i][c] = s / S[i][i];
        }
        (void)lo;
    }
    __syncthreads();
    // Z = L21 T11 (32 x 32), then T21 = -T22 Z
    for (int e = tid; e < 32 * 32; e += 256) {
        const int r = e / 32, c = e % 32;
        double s = 0.0;
        for (int q = c; q < 32; ++q) s += S[32 + r][q] * T[q][c];
        Z[r][c] = s;
    }
    __syncthreads();
    for (int e = tid; e < 32 * 32; e += 256) {
        const int r = e / 32, c = e % 32;
        double s = 0.0;
        for (int q = 0; q <= r; ++q) s += T[32 + r][32 + q] * Z[q][c];
        T[32 + r][c] = -s;
    }
    __syncthreads();
    double *Dk = D + (int64_t)k * kCb * kCb;
    for (int e = tid; e < kCb * kCb; e += 256) {
        const int r = e / kCb, c = e % kCb;
        Akk[(int64_t)r * N + c] = S[r][c];  // L_kk (zeros above the diagonal)
        Dk[e] = T[r][c];
    }
}

enum { kTilePanel = 0, kTileUpdate = 1, kTileInvRow = 2, kTileInvUpd = 3 };

// row r of the lower triangle (r >= c) holding linear index t of an m x m triangle
__device__ __forceinline__ void tri_index(int64_t t, int &r, int &c) {
    int64_t rr = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while (rr * (rr + 1) / 2 > t) --rr;
    while ((rr + 1) * (rr + 2) / 2 <= t) ++rr;
    r = (int)rr;
    c = (int)(t - rr * (rr + 1) / 2);
}

template <int MODE>
__global__ void __launch_bounds__(256) k_tile_mm(int64_t N, int nb, int k, double *__restrict__ A,
                                                 double *__restrict__ W, const double *__restrict__ D) {
    __shared__ double Xs[kCb][kCb + 1];  // Xs[row][kk]
    __shared__ double Ys[kCb][kCb + 1];  // Ys[kk][col]
    typedef double d4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t = blockIdx.x;
    int bi = 0, bj = 0;
    const double *X;
    const double *Y;
    int64_t ldx = N, ldy = N;
    bool yT = false;
    double *C;
    const double *Dk = D + (int64_t)k * kCb * kCb;
    if (MODE == kTilePanel) {
        bi = k + 1 + (int)t;
        bj = k;
        X = A + (int64_t)bi * kCb * N + (int64_t)k * kCb;
        Y = Dk;  // Y = D_k^T
        ldy = kCb;
        yT = true;
        C = A + (int64_t)bi * kCb * N + (int64_t)k * kCb;
    } else if (MODE == kTileUpdate) {
        int r, c;
        tri_index(t, r, c);
        bi = k + 1 + r;
        bj = k + 1 + c;
        X = A + (int64_t)bi * kCb * N + (int64_t)k * kCb;
        Y = A + (int64_t)bj * kCb * N + (int64_t)k * kCb;  // Y = A_jk^T
        yT = true;
        C = A + (int64_t)bi * kCb * N + (int64_t)bj * kCb;
    } else if (MODE == kTileInvRow) {
        bi = k;
        bj = (int)t;
        X = Dk;
        ldx = kCb;
        Y = W + (int64_t)k * kCb * N + (int64_t)bj * kCb;
        C = W + (int64_t)k * kCb * N + (int64_t)bj * kCb;
    } else {
        bi = k + 1 + (int)(t / (k + 1));
        bj = (int)(t % (k + 1));
        X = A + (int64_t)bi * kCb * N + (int64_t)k * kCb;
        Y = W + (int64_t)k * kCb * N + (int64_t)bj * kCb;
        C = W + (int64_t)bi * kCb * N + (int64_t)bj * kCb;
    }
    for (int e = tid; e < kCb * kCb; e += 256) {
        const int r = e / kCb, c = e % kCb;
        Xs[r][c] = X[(int64_t)r * ldx + c];
        const double yv = Y[(int64_t)r * ldy + c];
        if (yT) Ys[c][r] = yv;
        else Ys[r][c] = yv;
    }
    __syncthreads();
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    d4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < kCb / 4; ++s) {
        const int kk = s * 4 + (lane >> 4);
        double a[2], b[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = Xs[wr + i * 16 + (lane & 15)][kk];
#pragma unroll
        for (int j = 0; j < 2; ++j) b[j] = Ys[kk][wc + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    // C/D map of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = wr + i * 16 + (lane >> 4) + 4 * r;
                const int col = wc + j * 16 + (lane & 15);
                double *cp = C + (int64_t)row * N + col;
                const double v = acc[i][j][r];
                if (MODE == kTileUpdate || MODE == kTileInvUpd) *cp = *cp - v;
                else *cp = v;
            }
}

// Rank-(64 kb) tile updates, C -= sum_{q < kb} X_q Y_q over a tile region:
//   CHOL: C = A_ij, X_q = A_{i,k0+q}, Y_q = A_{j,k0+q}^T   (trailing lower triangle)
//   INV : C = W_ij, X_q = A_{i,k0+q}, Y_q = W_{k0+q,j}
// tri: tiles (i, j) with lo <= j <= i < hi; else i in [ilo, ihi), j in [jlo, jhi).
// Wider K (kb = 4: 256) reads and rewrites each C tile once per 4 block steps.
struct TileJob {
    int k0, kb;
    int ilo, ihi, jlo, jhi;
    int tri;
};

template <bool INV>
__global__ void __launch_bounds__(256) k_tile_upd(int64_t N, TileJob J, double *__restrict__ A,
                                                  double *__restrict__ W) {
    __shared__ double Xs[kCb][kCb + 1];
    __shared__ double Ys[kCb][kCb + 1];
    typedef double d4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t = blockIdx.x;
    int bi, bj;
    if (J.tri) {
        int r, c;
        tri_index(t, r, c);
        bi = J.ilo + r;
        bj = J.ilo + c;
    } else {
        const int w = J.jhi - J.jlo;
        bi = J.ilo + (int)(t / w);
        bj = J.jlo + (int)(t % w);
    }
    double *C = (INV ? W : A) + (int64_t)bi * kCb * N + (int64_t)bj * kCb;
    const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
    d4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = d4{0.0, 0.0, 0.0, 0.0};
    for (int q = 0; q < J.kb; ++q) {
        const int kq = J.k0 + q;
        const double *X = A + (int64_t)bi * kCb * N + (int64_t)kq * kCb;
        const double *Y = INV ? W + (int64_t)kq * kCb * N + (int64_t)bj * kCb
                              : A + (int64_t)bj * kCb * N + (int64_t)kq * kCb;
        for (int e = tid; e < kCb * kCb; e += 256) {
            const int r = e / kCb, c = e % kCb;
            Xs[r][c] = X[(int64_t)r * N + c];
            const double yv = Y[(int64_t)r * N + c];
            if (INV) Ys[r][c] = yv;
            else Ys[c][r] = yv;
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kCb / 4; ++s) {
            const int kk = s * 4 + (lane >> 4);
            double a[2], b[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = Xs[wr + i * 16 + (lane & 15)][kk];
#pragma unroll
            for (int j = 0; j < 2; ++j) b[j] = Ys[kk][wc + j * 16 + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = wr + i * 16 + (lane >> 4) + 4 * r;
                const int col = wc + j * 16 + (lane & 15);
                double *cp = C + (int64_t)row * N + col;
                *cp = *cp - acc[i][j][r];
            }
}

static unsigned tile_count(const TileJob &J) {
    if (J.tri) {
        const int64_t m = J.ihi - J.ilo;
        return (unsigned)(m * (m + 1) / 2);
    }
    return (unsigned)((int64_t)(J.ihi - J.ilo) * (J.jhi - J.jlo));
}

// U = W^T (64 x 64 tiles through LDS)
__global__ void __launch_bounds__(256) k_er_transpose(int64_t N, const double *__restrict__ W,
                                                      double *__restrict__ U) {
    __shared__ double T[kCb][kCb + 1];
    const int64_t nb = N / kCb;
    const int64_t bi = blockIdx.x / nb, bj = blockIdx.x % nb;
    for (int e = threadIdx.x; e < kCb * kCb; e += 256) {
        const int r = e / kCb, c = e % kCb;
        T[r][c] = W[(bi * kCb + r) * N + bj * kCb + c];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kCb * kCb; e += 256) {
        const int r = e / kCb, c = e % kCb;
        U[(bj * kCb + r) * N + bi * kCb + c] = T[c][r];
    }
}

// g[u] = G_uu = sum_{k >= u} U_uk^2, one wave per row
__global__ void __launch_bounds__(256) k_er_gdiag(int64_t n, int64_t N, const double *__restrict__ U,
                                                  double *__restrict__ g) {
    const int64_t u = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (u >= n) return;
    double s = 0.0;
    for (int64_t k = u + lane; k < N; k += 64) {
        const double x = U[u * N + k];
        s += x * x;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) g[u] = s;
}

// r_eff in CSR order, one wave per entry: G_uv = sum_{k >= max(u,v)} U_uk U_vk
__global__ void __launch_bounds__(256) k_er_chol_scores(int64_t N, const int32_t *__restrict__ rows,
                                                        const int32_t *__restrict__ ix, int64_t nnz,
                                                        const uint8_t *__restrict__ flag,
                                                        const double *__restrict__ U,
                                                        const double *__restrict__ g,
                                                        double *__restrict__ out) {
    const int64_t e = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (e >= nnz) return;
    const int64_t u = rows[e], v = ix[e];
    const bool fu = flag[u], fv = flag[v];
    double s = 0.0;
    if (!fu && !fv) {
        const int64_t k0 = u > v ? u : v;
        for (int64_t k = k0 + lane; k < N; k += 64) s += U[u * N + k] * U[v * N + k];
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (lane == 0) {
        const double guu = fu ? 0.0 : g[u];
        const double gvv = fv ? 0.0 : g[v];
        const double guv = (fu || fv) ? 0.0 : s;
        const double r = (guu + gvv) - 2.0 * guv;
        out[e] = r > 1e-10 ? r : 1e-10;
    }
}

// Connected components of the resident graph: label = smallest node id of the
// component (min-label propagation with pointer jumping); device buffer.
int32_t *components(gs_ctx *c) {
    Graph &g = c->g;
    hipStream_t st = c->stream;
    const int64_t n = g.n, nnz = g.nnz;
    auto *flags = (int *)c->buf("cc_flags").ensure(64);
    auto *lab = (int32_t *)c->buf("xer_lab").ensure(4 * (n ? n : 1));
    if (!n) return lab;
    k_cc_init<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, lab);
    for (int round = 0; round < 4096; ++round) {
        GS_HIP(hipMemsetAsync(flags, 0, 4, st));
        if (nnz)
            k_cc_hook<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(g.rows.as<int32_t>(),
                                                                g.indices.as<int32_t>(), nnz, lab,
                                                                flags);
        k_cc_jump<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, lab);
        int ch = 0;
        GS_HIP(hipMemcpyAsync(&ch, flags, 4, hipMemcpyDeviceToHost, st));
        GS_HIP(hipStreamSynchronize(st));
        if (!ch) break;
    }
    return lab;
}

// U = W^T for an N x N matrix (N a multiple of 64)
void transpose_square(gs_ctx *c, int64_t N, const double *W, double *U) {
    const int64_t nb = N / kCb;
    k_er_transpose<<<(unsigned)(nb * nb), 256, 0, c->stream>>>(N, W, U);
    GS_HIP(hipGetLastError());
}

// W = L^{-1} for the grounded M of the resident graph (identity rows where
// flag is set), M = L L^T by the blocked Cholesky of k_chol_diag / k_tile_mm /
// k_tile_upd; A and W are N x N scratch (A ends holding L).
void grounded_inverse(gs_ctx *c, int64_t N, const uint8_t *flag, double *A, double *W) {
    Graph &g = c->g;
    hipStream_t st = c->stream;
    const int64_t n = g.n;
    const size_t mb = sizeof(double) * (size_t)N * (size_t)N;
    const int64_t *ip = g.indptr.as<int64_t>();
    const int32_t *ix = g.indices.as<int32_t>();
    const double *dd = g.data.as<double>();
    auto *flags = (int *)c->buf("chol_flags").ensure(64);
    const int nb = (int)(N / kCb);
    double *D = (double *)c->buf("xer_D").ensure(sizeof(double) * (size_t)nb * kCb * kCb);
    GS_HIP(hipMemsetAsync(flags, 0, 4, st));
    GS_HIP(hipMemsetAsync(A, 0, mb, st));
    k_er_dense_rows<<<grid_for(N, 256, 8192), 256, 0, st>>>(n, N, ip, ix, dd, flag, A);
    double fl_upd = 0.0;
    const double tf = 2.0 * kCb * kCb * kCb;  // flops of one 64^3 tile product
    // block columns per panel: the trailing update runs at K = 64 P and rewrites
    // each C tile once per P block steps (Roman-like n = 22,662: P = 1 0.59 s,
    // 2 0.47 s, 4 0.39 s, 8 0.37 s)
    int P = 8;
    if (const char *e = getenv("GSPARSE_XER_PANEL")) P = atoi(e) >= 1 && atoi(e) <= 16 ? atoi(e) : 8;
    auto upd = [&](bool inv, const TileJob &J) {
        const unsigned cnt = tile_count(J);
        if (!cnt || J.kb <= 0) return;
        if (inv) k_tile_upd<true><<<cnt, 256, 0, st>>>(N, J, A, W);
        else k_tile_upd<false><<<cnt, 256, 0, st>>>(N, J, A, W);
        fl_upd += tf * J.kb * (double)cnt;
    };
    hipEvent_t t0 = prof_begin(c);
    for (int k0 = 0; k0 < nb; k0 += P) {
        const int kend = k0 + P < nb ? k0 + P : nb;
        for (int k = k0; k < kend; ++k) {
            k_chol_diag<<<1, 256, 0, st>>>(N, k, A, D, flags);
            const int m = nb - 1 - k;
            if (m > 0) {
                k_tile_mm<kTilePanel><<<(unsigned)m, 256, 0, st>>>(N, nb, k, A, W, D);
                fl_upd += tf * m;
            }
            // the panel's own later columns (i >= j, k < j < kend), one K = 64 step
            for (int j = k + 1; j < kend; ++j) upd(false, TileJob{k, 1, j, nb, j, j + 1, 0});
        }
        // the trailing lower triangle, K = 64 (kend - k0)
        upd(false, TileJob{k0, kend - k0, kend, nb, kend, nb, 1});
    }
    GS_HIP(hipMemsetAsync(W, 0, mb, st));
    k_er_identity<<<grid_for(N, 256, 8192), 256, 0, st>>>(N, W);
    for (int k0 = 0; k0 < nb; k0 += P) {
        const int kend = k0 + P < nb ? k0 + P : nb;
        for (int k = k0; k < kend; ++k) {
            k_tile_mm<kTileInvRow><<<(unsigned)(k + 1), 256, 0, st>>>(N, nb, k, A, W, D);
            fl_upd += tf * (k + 1);
            // rows of the panel below k (W_ij -= L_ik W_kj, j <= k)
            upd(true, TileJob{k, 1, k + 1, kend, 0, k + 1, 0});
        }
        // rows below the panel: W_ij -= sum_{k in panel} L_ik W_kj, j < kend
        upd(true, TileJob{k0, kend - k0, kend, nb, 0, kend, 0});
    }
    // the factorisation + inverse as one profiled region (flops executed on MFMA)
    prof_end(c, t0, "exact_er_dgemm", fl_upd);
    int bad = 0;
    GS_HIP(hipMemcpyAsync(&bad, flags, 4, hipMemcpyDeviceToHost, st));
    GS_HIP(hipStreamSynchronize(st));
    GS_CHECK(!bad, GS_EHIP, "Cholesky: non-positive pivot (M not positive definite)");
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
        const int64_t N = ((n + kGemmPad - 1) / kGemmPad) * kGemmPad;
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
            int32_t *lab = components(c);
            const int64_t *ip = g.indptr.as<int64_t>();
            const int32_t *ix = g.indices.as<int32_t>();
            const double *dd = g.data.as<double>();
            auto *best = (unsigned long long *)c->buf("xer_best").ensure(8 * n);
            auto *flag = (uint8_t *)c->buf("xer_flag").ensure(N);
            auto *mx = (unsigned long long *)c->buf("xer_mx").ensure(64);
            GS_HIP(hipMemsetAsync(best, 0, 8 * n, st));
            GS_HIP(hipMemsetAsync(mx, 0, 64, st));
            k_er_ground_pick<<<grid_for(n, 256, 8192), 256, 0, st>>>(n, ip, lab, best);
            k_er_ground_mark<<<grid_for(N, 256, 8192), 256, 0, st>>>(n, N, lab, best, flag);
            k_er_rownorm<<<grid_for(n, 256, 2048), 256, 0, st>>>(n, ip, ix, dd, flag, mx);
            const size_t mb = sizeof(double) * (size_t)N * (size_t)N;
            const char *meth = getenv("GSPARSE_XER_METHOD");
            if (!meth || strcmp(meth, "ns") != 0) {
                // blocked Cholesky + triangular inverse (see k_chol_diag)
                const int nb = (int)(N / kCb);
                double *A = (double *)c->buf("xer_X").ensure(mb);
                double *W = (double *)c->buf("xer_S").ensure(mb);
                double *gd = (double *)c->buf("xer_g").ensure(sizeof(double) * (size_t)n);
                grounded_inverse(c, N, flag, A, W);
                k_er_transpose<<<(unsigned)((int64_t)nb * nb), 256, 0, st>>>(N, W, A);
                k_er_gdiag<<<(unsigned)((n + 3) / 4), 256, 0, st>>>(n, N, A, gd);
                if (nnz)
                    k_er_chol_scores<<<(unsigned)((nnz + 3) / 4), 256, 0, st>>>(
                        N, g.rows.as<int32_t>(), ix, nnz, flag, A, gd, dout);
                GS_HIP(hipGetLastError());
                it_done = nb;
            } else {
            double *X = (double *)c->buf("xer_X").ensure(mb);
            double *X2 = (double *)c->buf("xer_X2").ensure(mb);
            double *S = (double *)c->buf("xer_S").ensure(mb);
            const int64_t sblocks = N * ((N + 255) / 256);
            auto *rpart = (double *)c->buf("xer_resid").ensure(8 * (sblocks + 1));
            k_er_xinit<<<grid_for(N * N, 256, 65536), 256, 0, st>>>(N, mx, X);
            const bool sym = !getenv("GSPARSE_XER_FULL");
            const bool dbg = getenv("GSPARSE_XER_DEBUG") != nullptr;
            // 64-wide tiles (4 waves/SIMD); the 128-wide form holds 1 wave/SIMD and
            // measured slower at every size (DESIGN.md §Exact ER), kept behind the knob
            int tm = 64;
            if (const char *e = getenv("GSPARSE_XER_TILE")) tm = (atoi(e) == 128 && N % 128 == 0) ? 128 : 64;
            const int64_t nb = N / tm;
            const unsigned gg = (unsigned)(sym ? nb * (nb + 1) / 2 : nb * nb);
            // flops one launch executes (the symmetric form runs nb(nb+1)/2 of nb^2 tiles)
            const double flops = 2.0 * tm * tm * (double)N * (double)gg;
            // algorithmic bytes of S = M X: X row gathers per entry + X_i + S_i per row
            const double sbytes = 8.0 * (double)N * (double)(nnz + 2 * N);
            double prev = 1e300;
            for (int it = 0; it < 256; ++it) {
                hipEvent_t t0 = prof_begin(c);
                k_er_spmm<<<(unsigned)sblocks, 256, 0, st>>>(n, N, ip, ix, dd, flag, X, S, rpart);
                prof_end(c, t0, "exact_er_spmm", sbytes);
                k_er_resid_fin<<<1, 256, 0, st>>>(rpart, sblocks, rpart + sblocks);
                double res = 0.0;
                GS_HIP(hipMemcpyAsync(&res, rpart + sblocks, 8, hipMemcpyDeviceToHost, st));
                GS_HIP(hipStreamSynchronize(st));
                it_done = it;
                if (dbg) fprintf(stderr, "[gs_exact_er] it=%d residual=%.6e\n", it, res);
                GS_CHECK(std::isfinite(res), GS_EHIP, "Newton-Schulz diverged at step %d", it);
                // converged, or rounding has taken over: in the quadratic phase each
                // step squares the residual, at the rounding floor it stalls
                if (res < 1e-14 * (double)N || (prev < 1e-2 && res > 0.5 * prev)) break;
                GS_CHECK(it < 255, GS_EHIP, "Newton-Schulz did not converge (residual %g)", res);
                prev = res;
                t0 = prof_begin(c);
                // X2 = 2X - X S
                if (sym && tm == 128)
                    k_dgemm<true, 128><<<gg, 256, 0, st>>>(N, X, S, -1.0, 2.0, X, X2);
                else if (sym)
                    k_dgemm<true, 64><<<gg, 256, 0, st>>>(N, X, S, -1.0, 2.0, X, X2);
                else if (tm == 128)
                    k_dgemm<false, 128><<<gg, 256, 0, st>>>(N, X, S, -1.0, 2.0, X, X2);
                else
                    k_dgemm<false, 64><<<gg, 256, 0, st>>>(N, X, S, -1.0, 2.0, X, X2);
                prof_end(c, t0, "exact_er_dgemm", flops);
                std::swap(X, X2);
            }
            if (nnz)
                k_er_exact_scores<<<grid_for(nnz, 256, 8192), 256, 0, st>>>(
                    N, g.rows.as<int32_t>(), ix, nnz, flag, X, dout);
            GS_HIP(hipGetLastError());
            }
        }
        finish_out(c, out, dout, sizeof(double) * nnz, loc);
        if (iterations) *iterations = it_done;
    });
}
