// gs_er.hip -- ApproxER (calculate_approx_effective_resistance_scores,
// metrics.py:178-298) on the device, bit-exact with the reference.
//
// Layout in HBM (row-major n x k, the JL columns contiguous per node):
//   Rr  residual, initialised with Y = B @ R           (metrics.py:275)
//   X   solution, P0/P1 search direction (ping-pong), Q = L_reg p (whole in
//       modes 1-3, else only the leftover rows of each BLAS chunk)
// The k CG solves (metrics.py:284-289, SciPy 1.15 cg recurrence) run as one
// batched iteration.  Short rows (mode 0), two fused kernels per iteration:
//   k_cg_pq : x += fl(alpha_{t-1} p_{t-1}) (deferred x update of the previous
//             iteration); p = beta*p + r (two roundings), neighbours' p
//             recomputed; q = L_reg p (per-row fold from 0.0 in ascending
//             column, products rounded); partial dot(p,q)
//   k_cg_upd: q recomputed from the stored p; r -= fl(alpha q); partial dot(r,r)
// (64 B per entry and iteration).  Long rows (mode 3): k_cg_p_flat (p stream),
// k_spmv (column-block-major SpMV, q stored), k_dot_acc, k_cg_upd<STOREQ>.
// Plus two per-column finish kernels.  Every dot product reproduces
// OpenBLAS ddot (SkylakeX kernel) as np.dot calls it: T thread chunks for
// n > 10000, inside a chunk 32 FMA accumulator chains over rows j, j+32, ...,
// then the 32->16 fold, the optional 16-block, the 4-lane tree and the FMA
// tail (pinned in oracle.c, oracle_ddot).  A lane of k_cg_* owns one
// (column, chunk, residue j) chain: the chain IS the thread's row loop, so
// the reduction costs no extra pass over HBM.
#include "gs_internal.hpp"
#include "gs_pairwise.hpp"

namespace gs {

static constexpr int kMaxChunks = 64;
static constexpr int64_t kStoreQRowLen = 8;  // L_reg entries per row above which q is stored

struct Chunks {
    int32_t count;
    int64_t a[kMaxChunks];
    int64_t len[kMaxChunks];
};

static Chunks make_chunks(int64_t n, int32_t threads) {
    Chunks ch{};
    if (n <= 10000 || threads <= 1) {
        ch.count = 1;
        ch.a[0] = 0;
        ch.len[0] = n;
        return ch;
    }
    // OpenBLAS's own thread limit (MAX_THREADS=64 in NumPy's build): more threads
    // cannot occur in the reference and are refused in gs_er_solve
    int64_t lo = 0, rem = n;
    int32_t cnt = 0;
    for (int32_t t = threads; t > 0 && rem > 0; --t) {
        int64_t w = (rem + t - 1) / t;
        ch.a[cnt] = lo;
        ch.len[cnt] = w;
        ++cnt;
        lo += w;
        rem -= w;
    }
    ch.count = cnt;
    return ch;
}

// per-column state, structure of arrays inside one buffer
struct ColPtrs {
    double *bn, *atol, *rho, *rho_prev, *alpha;
    int32_t *active, *iters;
    int32_t *xstep;    // iteration whose (alpha, p) is still to be added to x
    int32_t *nactive;  // single counter
};

static ColPtrs col_ptrs(ErState &er) {
    int64_t k = er.k;
    char *b = (char *)er.colstate.ptr;
    ColPtrs p;
    p.bn = (double *)b;
    p.atol = p.bn + k;
    p.rho = p.atol + k;
    p.rho_prev = p.rho + k;
    p.alpha = p.rho_prev + k;
    p.active = (int32_t *)(p.alpha + k);
    p.iters = p.active + k;
    p.xstep = p.iters + k;
    p.nactive = p.xstep + k;
    return p;
}

// ---------------------------------------------------------------- prepare
__global__ void k_upper_flags(const int32_t *__restrict__ rows, const int32_t *__restrict__ ix,
                              int64_t nnz, int64_t *__restrict__ flag) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x)
        flag[e] = rows[e] < ix[e] ? 1 : 0;
}

__global__ void k_edge_ids(const int64_t *__restrict__ flag, const int64_t *__restrict__ pos,
                           int64_t nnz, int64_t *__restrict__ eid) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < nnz;
         e += (int64_t)gridDim.x * blockDim.x)
        eid[e] = flag[e] ? pos[e] : -1;
}

// B row counts: node i is incident to (u,i) u<i (transposed column i) and (i,j) j>i (row i).
__global__ void k_b_counts(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                           const int64_t *__restrict__ tp, const int32_t *__restrict__ ti,
                           int64_t n, int64_t *__restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t c = 0;
        for (int64_t t = tp[i]; t < tp[i + 1]; ++t) c += ti[t] < i;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e) c += ix[e] > i;
        cnt[i] = c;
    }
}

__global__ void k_b_fill(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                         const int64_t *__restrict__ tp, const int32_t *__restrict__ ti,
                         const int64_t *__restrict__ tpos, const int64_t *__restrict__ eid,
                         int64_t n, const int64_t *__restrict__ bptr, int64_t *__restrict__ bcol,
                         int8_t *__restrict__ bsgn, int64_t *__restrict__ bcur) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t o = bptr[i];
        bcur[i] = o;
        // (u, i) with u < i: edge ids ascending with u (row-major numbering), sign -1
        for (int64_t t = tp[i]; t < tp[i + 1]; ++t)
            if (ti[t] < i) {
                bcol[o] = eid[tpos[t]];
                bsgn[o] = -1;
                ++o;
            }
        // (i, j) with j > i: after every (u, i), sign +1
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e)
            if (ix[e] > i) {
                bcol[o] = eid[e];
                bsgn[o] = 1;
                ++o;
            }
    }
}

// L = diag(rowsum A) - A (zeros dropped, SciPy csr_minus), L_reg = L + reg I.
__device__ __forceinline__ void lrow_diag(const int64_t *ip, const int32_t *ix, const double *d,
                                          int64_t i, double reg, double &diag, bool &has_diag) {
    double deg = 0.0, aii = 0.0;
    bool self = false;
    for (int64_t e = ip[i]; e < ip[i + 1]; ++e) {
        deg = deg + d[e];  // adj.sum(axis=1): fold ascending column from 0.0
        if (ix[e] == i) {
            self = true;
            aii = d[e];
        }
    }
    // D_ii present iff deg != 0 (dia->csr drops zeros)
    bool has_l = false;
    double l = 0.0;
    if (deg != 0.0 && self) {
        l = deg - aii;
        has_l = l != 0.0;
    } else if (deg != 0.0) {
        l = deg;
        has_l = true;
    } else if (self) {
        l = 0.0 - aii;
        has_l = l != 0.0;
    }
    diag = has_l ? l + reg : reg;
    has_diag = diag != 0.0;
}

__global__ void k_l_counts(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                           const double *__restrict__ d, int64_t n, double reg,
                           int64_t *__restrict__ cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double dg;
        bool hd;
        lrow_diag(ip, ix, d, i, reg, dg, hd);
        int64_t c = hd ? 1 : 0;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e)
            if (ix[e] != i && d[e] != 0.0) ++c;
        cnt[i] = c;
    }
}

__global__ void k_l_fill(const int64_t *__restrict__ ip, const int32_t *__restrict__ ix,
                         const double *__restrict__ d, int64_t n, double reg,
                         const int64_t *__restrict__ lp, int32_t *__restrict__ li,
                         double *__restrict__ lv) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double dg;
        bool hd;
        lrow_diag(ip, ix, d, i, reg, dg, hd);
        int64_t o = lp[i];
        bool placed = !hd;
        for (int64_t e = ip[i]; e < ip[i + 1]; ++e) {
            int32_t j = ix[e];
            if (!placed && j >= i) {
                li[o] = (int32_t)i;
                lv[o] = dg;
                ++o;
                placed = true;
            }
            if (j != i && d[e] != 0.0) {
                li[o] = j;
                lv[o] = 0.0 - d[e];
                ++o;
            }
        }
        if (!placed) {
            li[o] = (int32_t)i;
            lv[o] = dg;
        }
    }
}

// ---------------------------------------------------------------- projection
// Y[i,c] += sign * raw[e - e0, c - rc0] / sqrt_k for node i's incident edges e in
// [e0, e1), in ascending e (metrics.py:272-275; SciPy csr_matvecs folds B's
// sorted row from 0.0, +-1 * R exact), for the columns c in [c0, c1).  One wave per
// node and 64-column slice.  raw is row-major with stride kraw, its column 0 being
// Y's column rc0 (NumPy's whole rows: kraw = k, rc0 = 0; a rank's slice: kraw =
// c1 - c0, rc0 = c0); Y has stride ld.  The first rows (e0 == 0) fold from 0.0,
// later row chunks from the Y the earlier ones left.
__global__ void __launch_bounds__(256) k_project(const int64_t *__restrict__ bptr,
                                                 const int64_t *__restrict__ bcol,
                                                 const int8_t *__restrict__ bsgn, int64_t n,
                                                 int64_t c0, int64_t c1, int64_t kraw, int64_t rc0,
                                                 int64_t ld, int64_t e0, int64_t e1,
                                                 const double *__restrict__ raw, double sqrt_k,
                                                 double *__restrict__ Y) {
    const int64_t k = c1;
    int64_t ncb = (c1 - c0 + 63) / 64;
    int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
    int lane = threadIdx.x & 63;
    int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t w = wave; w < n * ncb; w += nwaves) {
        int64_t i = w / ncb, cb = w % ncb;
        int64_t c = c0 + cb * 64 + lane;
        // first incident edge id >= e0 (B rows are sorted): stateless, so the
        // column slices of one node need no shared cursor
        int64_t p = bptr[i], end = bptr[i + 1];
        {
            int64_t hi = end;
            while (p < hi) {
                int64_t mid = (p + hi) >> 1;
                if (bcol[mid] < e0) p = mid + 1;
                else hi = mid;
            }
        }
        double y = (c < k && e0 > 0) ? Y[i * ld + c] : 0.0;
        for (; p < end; ++p) {
            int64_t e = bcol[p];
            if (e >= e1) break;
            if (c < k) {
                double r = raw[(e - e0) * kraw + (c - rc0)] / sqrt_k;
                double t = bsgn[p] > 0 ? r : -r;
                y = y + t;
            }
        }
        if (c < k) Y[i * ld + c] = y;
    }
}

// ---------------------------------------------------------------- CG kernels
struct ChunkArg {
    int32_t count;
    int64_t a[kMaxChunks];
    int64_t len[kMaxChunks];
};

// Geometry of one batched-CG launch.  Lane layout: a wave owns ONE residue
// j (rows j, j+32, ... of a BLAS chunk -- that row sequence IS the OpenBLAS
// accumulator chain j) for CPL*64 consecutive columns, CPL columns per lane
// (CPL=2: 16-byte loads, two independent chains per lane).  A 256-thread
// workgroup holds 4 residues; the 8 workgroups of one (column block, chunk)
// pair get block ids b, b+8, ..., b+56 -- under the round-robin dispatch over
// the 8 XCDs they share one XCD's L2, so the neighbour rows a chain's SpMV
// gathers (mostly rows i-1, i+1, i+chord: other residues) are L2 hits.
struct CgGeom {
    int64_t n, k, ld, col0, col1;
    int32_t ncb;     // column blocks of CPL*64
    int32_t npairs;  // ncb * chunks
};

struct CgLane {
    int64_t c;   // first column of this lane
    int j, t;    // residue, chunk
    bool ok;
};

template <int CPL>
__device__ __forceinline__ CgLane cg_lane(const CgGeom &G) {
    const int b = blockIdx.x;
    const int grp = b >> 6, r = b & 63;
    const int sub = r & 7, part = r >> 3;  // part: which 4 of the 32 residues
    const int pair = grp * 8 + sub;
    CgLane L;
    L.ok = pair < G.npairs;
    const int cb = pair % G.ncb;
    L.t = pair / G.ncb;
    L.j = __builtin_amdgcn_readfirstlane(part * 4 + (int)(threadIdx.x >> 6));
    L.c = G.col0 + (int64_t)cb * (64 * CPL) + (int64_t)(threadIdx.x & 63) * CPL;
    return L;
}

template <int CPL>
struct Vec;
template <>
struct Vec<1> {
    double v[1];
    __device__ __forceinline__ void load(const double *p) { v[0] = *p; }
    __device__ __forceinline__ void store(double *p) const { *p = v[0]; }
};
template <>
struct Vec<2> {
    double v[2];
    __device__ __forceinline__ void load(const double *p) {
        double2 t = *reinterpret_cast<const double2 *>(p);
        v[0] = t.x;
        v[1] = t.y;
    }
    __device__ __forceinline__ void store(double *p) const {
        *reinterpret_cast<double2 *>(p) = make_double2(v[0], v[1]);
    }
};

// Iteration t, kernel 1 (after beta_t is known):
//   x += fl(alpha_{t-1} p_{t-1})   for columns whose previous update is pending
//                                  (the x update of SciPy's iteration t-1, moved
//                                  here so the second kernel never touches x or p)
//   p_t = fl(fl(beta_t p_{t-1}) + r_t)  (own row stored; neighbours recomputed)
//   q_t = L_reg p_t (per-row fold from 0.0, ascending column), kept only for the
//         <32 leftover rows the ddot finish needs (qside); chains of dot(p_t, q_t).
template <bool FIRST, int CPL, bool STOREQ, int RU>
__global__ void __launch_bounds__(256) k_cg_pq(CgGeom G, ChunkArg ch,
                                               const int64_t *__restrict__ lp,
                                               const int32_t *__restrict__ li,
                                               const double *__restrict__ lv,
                                               const double *__restrict__ R,
                                               const double *__restrict__ Pold,
                                               double *__restrict__ Pnew, double *__restrict__ X,
                                               double *__restrict__ qside,
                                               double *__restrict__ Q,
                                               const double *__restrict__ rho,
                                               const double *__restrict__ rho_prev,
                                               const double *__restrict__ alpha,
                                               const int32_t *__restrict__ active,
                                               const int32_t *__restrict__ xstep, int32_t it,
                                               double *__restrict__ acc) {
    const CgLane ln = cg_lane<CPL>(G);
    if (!ln.ok) return;
    const int64_t ld = G.ld, c = ln.c;
    bool live[CPL], xp[CPL];
    double beta[CPL], al[CPL];
    bool any_live = false, any_x = false;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        const bool in = (c + u) < G.col1;
        live[u] = in && active[c + u];
        xp[u] = !FIRST && in && xstep[c + u] == it - 1;
        beta[u] = (!FIRST && live[u]) ? rho[c + u] / rho_prev[c + u] : 0.0;
        al[u] = xp[u] ? alpha[c + u] : 0.0;
        any_live = any_live || live[u];
        any_x = any_x || xp[u];
    }
    if (!any_live && !any_x) return;
    const int64_t a = ch.a[ln.t], L = ch.len[ln.t];
    const int64_t n1 = L & ~(int64_t)15, n32 = n1 & ~(int64_t)31;
    double s[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) s[u] = 0.0;

    // RU rows of the chain per trip (rows ok[i]; ok[0] always holds).  The trip
    // is branch-free up to the stores: absent rows and entries past a row's
    // end load from valid addresses (row[0], the row's last entry) and are
    // masked by selects, so every load of a step is in flight at once.
    auto rows_pq = [&](const int64_t *row, const bool *ok, double (*pi)[CPL], double (*q)[CPL]) {
        int64_t rc[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) rc[i] = ok[i] ? row[i] : row[0];
        Vec<CPL> po[RU], xv[RU];
        if (!FIRST && any_x) {
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                po[i].load(Pold + rc[i] * ld + c);
                xv[i].load(X + rc[i] * ld + c);
            }
        }
        int64_t e0[RU], len[RU], maxlen = 0;
        bool found[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            e0[i] = lp[rc[i]];
            const int64_t e1 = lp[rc[i] + 1];  // unconditional: keeps the loads of all rows in flight
            len[i] = ok[i] ? e1 - e0[i] : 0;
            maxlen = len[i] > maxlen ? len[i] : maxlen;
            found[i] = false;
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                q[i][u] = 0.0;
                pi[i][u] = 0.0;
            }
        }
        if (!any_live) maxlen = 0;
        for (int64_t k = 0; k < maxlen; ++k) {
            int32_t col[RU];
            double w[RU];
            Vec<CPL> rv[RU], pv[RU];
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                const int64_t kk = k < len[i] ? k : (len[i] > 0 ? len[i] - 1 : 0);
                col[i] = li[e0[i] + kk];
                w[i] = lv[e0[i] + kk];
            }
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                rv[i].load(R + col[i] * ld + c);
                if (!FIRST) pv[i].load(Pold + col[i] * ld + c);
            }
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                const bool act = k < len[i];
                const bool diag = act && col[i] == row[i];
#pragma unroll
                for (int u = 0; u < CPL; ++u) {
                    double pn;
                    if (FIRST) {
                        pn = rv[i].v[u];
                    } else {
                        double pb = pv[i].v[u] * beta[u];
                        pn = pb + rv[i].v[u];
                    }
                    pi[i][u] = diag ? pn : pi[i][u];
                    double prod = w[i] * pn;
                    double qn = q[i][u] + prod;
                    q[i][u] = act ? qn : q[i][u];
                }
                found[i] = found[i] || diag;
            }
        }
        if (!FIRST && any_x) {
#pragma unroll
            for (int i = 0; i < RU; ++i)
                if (ok[i]) {
#pragma unroll
                    for (int u = 0; u < CPL; ++u)
                        if (xp[u]) {
                            double t1 = al[u] * po[i].v[u];
                            xv[i].v[u] = xv[i].v[u] + t1;
                        }
                    xv[i].store(X + row[i] * ld + c);
                }
        }
        if (!any_live) return;
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            if (!ok[i]) continue;
            if (!found[i]) {  // L_reg_ii dropped (== 0): p_i still needed
                Vec<CPL> rv, pv;
                rv.load(R + row[i] * ld + c);
                if (!FIRST) pv.load(Pold + row[i] * ld + c);
#pragma unroll
                for (int u = 0; u < CPL; ++u) {
                    if (FIRST) {
                        pi[i][u] = rv.v[u];
                    } else {
                        double pb = pv.v[u] * beta[u];
                        pi[i][u] = pb + rv.v[u];
                    }
                }
            }
            const int64_t o = row[i] * ld + c;
            Vec<CPL> pw;
#pragma unroll
            for (int u = 0; u < CPL; ++u) pw.v[u] = live[u] ? pi[i][u] : 0.0;
            // columns that are not live keep their last p (the flush may need it)
            if (CPL == 1 || (live[0] && live[CPL - 1])) {
                pw.store(Pnew + o);
            } else {
#pragma unroll
                for (int u = 0; u < CPL; ++u)
                    if (live[u]) Pnew[o + u] = pi[i][u];
            }
            if (STOREQ) {  // q kept, the update kernel streams it
                Vec<CPL> qw;
#pragma unroll
                for (int u = 0; u < CPL; ++u) qw.v[u] = q[i][u];
                if (CPL == 1 || (live[0] && live[CPL - 1])) {
                    qw.store(Q + o);
                } else {
#pragma unroll
                    for (int u = 0; u < CPL; ++u)
                        if (live[u]) Q[o + u] = q[i][u];
                }
            }
        }
    };

    for (int64_t base = a + ln.j; base < a + n32; base += 32 * RU) {
        int64_t row[RU];
        bool ok[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            row[i] = base + 32 * i;
            ok[i] = row[i] < a + n32;
        }
        double pi[RU][CPL], q[RU][CPL];
        rows_pq(row, ok, pi, q);
#pragma unroll
        for (int i = 0; i < RU; ++i)
            if (ok[i])
#pragma unroll
                for (int u = 0; u < CPL; ++u) s[u] = __builtin_fma(pi[i][u], q[i][u], s[u]);
    }
    {  // leftover rows of the chunk (16-block + tail): q kept for the finish
        int64_t row[RU];
        bool ok[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            row[i] = a + n32 + ln.j;
            ok[i] = i == 0 && row[i] < a + L;
        }
        if (ok[0]) {
            double pi[RU][CPL], q[RU][CPL];
            rows_pq(row, ok, pi, q);
            if (!STOREQ && any_live) {
                double *qs = qside + ((int64_t)ln.t * 32 + ln.j) * ld + c;
#pragma unroll
                for (int u = 0; u < CPL; ++u)
                    if (live[u]) qs[u] = q[0][u];
            }
        }
    }
    if (any_live) {
#pragma unroll
        for (int u = 0; u < CPL; ++u)
            if (live[u]) acc[((c + u - G.col0) * kMaxChunks + ln.t) * 32 + ln.j] = s[u];
    }
}

// Iteration t, kernel 2 (after alpha_t is known):
//   q_t = L_reg p_t recomputed from the stored p_t (same fold, same bits) or
//   read (STOREQ), r_{t+1} = r_t - fl(alpha_t q_t); chains of dot(r_{t+1}, r_{t+1}).
template <int CPL, bool STOREQ, int RU>
__global__ void __launch_bounds__(256) k_cg_upd(CgGeom G, ChunkArg ch,
                                                const int64_t *__restrict__ lp,
                                                const int32_t *__restrict__ li,
                                                const double *__restrict__ lv,
                                                const double *__restrict__ P,
                                                const double *__restrict__ Q,
                                                double *__restrict__ R,
                                                const double *__restrict__ alpha,
                                                const int32_t *__restrict__ active,
                                                double *__restrict__ acc) {
    const CgLane ln = cg_lane<CPL>(G);
    if (!ln.ok) return;
    const int64_t ld = G.ld, c = ln.c;
    double al[CPL];
    bool live[CPL];
    bool any = false;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        live[u] = (c + u) < G.col1 && active[c + u];
        al[u] = live[u] ? alpha[c + u] : 0.0;
        any = any || live[u];
    }
    if (!any) return;
    const int64_t a = ch.a[ln.t], L = ch.len[ln.t];
    const int64_t n1 = L & ~(int64_t)15, n32 = n1 & ~(int64_t)31;
    double s[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) s[u] = 0.0;
    auto rows_upd = [&](const int64_t *row, const bool *ok, Vec<CPL> *rv) {
        double q[RU][CPL];
        int64_t rc[RU], e0[RU], len[RU], maxlen = 0;
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            rc[i] = ok[i] ? row[i] : row[0];
            rv[i].load(R + rc[i] * ld + c);
#pragma unroll
            for (int u = 0; u < CPL; ++u) q[i][u] = 0.0;
            if (STOREQ) {
                Vec<CPL> qv;
                qv.load(Q + rc[i] * ld + c);
#pragma unroll
                for (int u = 0; u < CPL; ++u) q[i][u] = qv.v[u];
            }
            e0[i] = STOREQ ? 0 : lp[rc[i]];
            const int64_t e1 = STOREQ ? 0 : lp[rc[i] + 1];
            len[i] = (!STOREQ && ok[i]) ? e1 - e0[i] : 0;
            maxlen = len[i] > maxlen ? len[i] : maxlen;
        }
        for (int64_t k = 0; k < maxlen; ++k) {
            double w[RU];
            Vec<CPL> pv[RU];
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                const int64_t kk = k < len[i] ? k : (len[i] > 0 ? len[i] - 1 : 0);
                const int32_t col = li[e0[i] + kk];
                w[i] = lv[e0[i] + kk];
                pv[i].load(P + col * ld + c);
            }
#pragma unroll
            for (int i = 0; i < RU; ++i) {
                const bool act = k < len[i];
#pragma unroll
                for (int u = 0; u < CPL; ++u) {
                    double prod = w[i] * pv[i].v[u];
                    double qn = q[i][u] + prod;
                    q[i][u] = act ? qn : q[i][u];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < RU; ++i)
            if (ok[i]) {
#pragma unroll
                for (int u = 0; u < CPL; ++u) {
                    double t2 = al[u] * q[i][u];
                    rv[i].v[u] = live[u] ? rv[i].v[u] - t2 : rv[i].v[u];
                }
                rv[i].store(R + row[i] * ld + c);
            }
    };
    for (int64_t base = a + ln.j; base < a + n32; base += 32 * RU) {
        int64_t row[RU];
        bool ok[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            row[i] = base + 32 * i;
            ok[i] = row[i] < a + n32;
        }
        Vec<CPL> rv[RU];
        rows_upd(row, ok, rv);
#pragma unroll
        for (int i = 0; i < RU; ++i)
            if (ok[i])
#pragma unroll
                for (int u = 0; u < CPL; ++u) s[u] = __builtin_fma(rv[i].v[u], rv[i].v[u], s[u]);
    }
    {
        int64_t row[RU];
        bool ok[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            row[i] = a + n32 + ln.j;
            ok[i] = i == 0 && row[i] < a + L;
        }
        if (ok[0]) {
            Vec<CPL> rv[RU];
            rows_upd(row, ok, rv);
        }
    }
#pragma unroll
    for (int u = 0; u < CPL; ++u)
        if (live[u]) acc[((c + u - G.col0) * kMaxChunks + ln.t) * 32 + ln.j] = s[u];
}

// Split modes (rows with many entries, where recomputing a neighbour's p costs
// two gathers, or few columns, where the chains give too few waves):
//   k_cg_p_flat : x += fl(alpha_{t-1} p_{t-1}) (pending columns); p_t = fl(fl(beta p) + r)
//   k_cg_q (mode 2) : q_t = L_reg p_t (gathers of the stored p), q stored, dot(p, q) chains
//   k_spmv + k_dot_acc (mode 3) : the same, SpMV in column-block-major order
//   k_cg_upd<STOREQ> : r -= fl(alpha q) streaming q
// The p update has no reduction, so it streams flat: threads own a column pair
// (16 B, flags loaded once), blockIdx.y a band of kFlatRows rows, rows
// walked in order -- each wave reads 1 KB contiguous per row.
static constexpr int kFlatRows = 16;

template <bool FIRST>
__global__ void __launch_bounds__(256) k_cg_p_flat(CgGeom G, const double *__restrict__ R,
                                                   const double *__restrict__ Pold,
                                                   double *__restrict__ Pnew,
                                                   double *__restrict__ X,
                                                   const double *__restrict__ rho,
                                                   const double *__restrict__ rho_prev,
                                                   const double *__restrict__ alpha,
                                                   const int32_t *__restrict__ active,
                                                   const int32_t *__restrict__ xstep, int32_t it) {
    const int64_t c = G.col0 + 2 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
    if (c >= G.col1) return;
    bool live[2], xp[2];
    double beta[2], al[2];
    bool any_live = false, any_x = false;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const bool in = (c + u) < G.col1;
        live[u] = in && active[c + u];
        xp[u] = !FIRST && in && xstep[c + u] == it - 1;
        beta[u] = (!FIRST && live[u]) ? rho[c + u] / rho_prev[c + u] : 0.0;
        al[u] = xp[u] ? alpha[c + u] : 0.0;
        any_live = any_live || live[u];
        any_x = any_x || xp[u];
    }
    if (!any_live && !any_x) return;
    const int64_t r0 = (int64_t)blockIdx.y * kFlatRows;
    const int64_t r1 = r0 + kFlatRows < G.n ? r0 + kFlatRows : G.n;
    for (int64_t row = r0; row < r1; ++row) {
        const int64_t o = row * G.ld + c;
        Vec<2> po, rv, xv;
        if (!FIRST) po.load(Pold + o);
        if (any_x) xv.load(X + o);
        if (any_live) rv.load(R + o);
        if (any_x) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (xp[u]) {
                    double t1 = al[u] * po.v[u];
                    xv.v[u] = xv.v[u] + t1;
                }
            if (xp[0] && xp[1]) xv.store(X + o);
            else
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    if (xp[u]) X[o + u] = xv.v[u];
        }
        if (!any_live) continue;
        Vec<2> pw;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            double pn;
            if (FIRST) {
                pn = rv.v[u];
            } else {
                double pb = po.v[u] * beta[u];
                pn = pb + rv.v[u];
            }
            pw.v[u] = pn;
        }
        if (live[0] && live[1]) pw.store(Pnew + o);
        else
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (live[u]) Pnew[o + u] = pw.v[u];
    }
}

template <int CPL>
__global__ void __launch_bounds__(256) k_cg_q(CgGeom G, ChunkArg ch, const int64_t *__restrict__ lp,
                                              const int32_t *__restrict__ li,
                                              const double *__restrict__ lv,
                                              const double *__restrict__ P,
                                              double *__restrict__ Q,
                                              const int32_t *__restrict__ active,
                                              double *__restrict__ acc) {
    const CgLane ln = cg_lane<CPL>(G);
    if (!ln.ok) return;
    const int64_t ld = G.ld, c = ln.c;
    bool live[CPL];
    bool any = false;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        live[u] = (c + u) < G.col1 && active[c + u];
        any = any || live[u];
    }
    if (!any) return;
    const int64_t a = ch.a[ln.t], L = ch.len[ln.t];
    const int64_t n1 = L & ~(int64_t)15, n32 = n1 & ~(int64_t)31;
    double s[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) s[u] = 0.0;
    auto row_q = [&](int64_t row, double *pi, double *q) {
        const int64_t e0 = lp[row], e1 = lp[row + 1];
        bool found = false;
#pragma unroll
        for (int u = 0; u < CPL; ++u) q[u] = 0.0;
        for (int64_t e = e0; e < e1; ++e) {
            const int32_t col = li[e];
            const double w = lv[e];
            Vec<CPL> pv;
            pv.load(P + col * ld + c);
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                if (col == row) pi[u] = pv.v[u];
                double prod = w * pv.v[u];
                q[u] = q[u] + prod;
            }
            found = found || (col == row);
        }
        if (!found) {  // L_reg_ii dropped (== 0): p_i still needed
            Vec<CPL> pv;
            pv.load(P + row * ld + c);
#pragma unroll
            for (int u = 0; u < CPL; ++u) pi[u] = pv.v[u];
        }
        Vec<CPL> qw;
#pragma unroll
        for (int u = 0; u < CPL; ++u) qw.v[u] = q[u];
        if (CPL == 1 || (live[0] && live[CPL - 1])) {
            qw.store(Q + row * ld + c);
        } else {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
                if (live[u]) Q[row * ld + c + u] = q[u];
        }
    };
    for (int64_t row = a + ln.j; row < a + n32; row += 32) {
        double pi[CPL], q[CPL];
        row_q(row, pi, q);
#pragma unroll
        for (int u = 0; u < CPL; ++u) s[u] = __builtin_fma(pi[u], q[u], s[u]);
    }
    {
        const int64_t row = a + n32 + ln.j;
        if (row < a + L) {
            double pi[CPL], q[CPL];
            row_q(row, pi, q);
        }
    }
#pragma unroll
    for (int u = 0; u < CPL; ++u)
        if (live[u]) acc[((c + u - G.col0) * kMaxChunks + ln.t) * 32 + ln.j] = s[u];
}

// q = L_reg p with no reduction attached, so any row order is allowed: waves
// walk row tiles with the column block as the SLOWEST index, so the blocks in
// flight (n x 64*CPL doubles each) stay resident in the Infinity Cache while
// their rows are gathered.  dot(p, q) then comes from k_dot_acc.
template <int CPL>
__global__ void __launch_bounds__(256) k_spmv(CgGeom G, int64_t rpw, int64_t ntiles,
                                              const int64_t *__restrict__ lp,
                                              const int32_t *__restrict__ li,
                                              const double *__restrict__ lv,
                                              const double *__restrict__ P,
                                              double *__restrict__ Q,
                                              const int32_t *__restrict__ active) {
    const int64_t gw = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t cb = gw / ntiles, tile = gw % ntiles;
    if (cb >= G.ncb) return;
    const int64_t ld = G.ld, c = G.col0 + cb * (64 * CPL) + (int64_t)(threadIdx.x & 63) * CPL;
    bool live[CPL];
    bool any = false;
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
        live[u] = (c + u) < G.col1 && active[c + u];
        any = any || live[u];
    }
    if (!any) return;
    const int64_t r0 = tile * rpw, r1 = r0 + rpw < G.n ? r0 + rpw : G.n;
    for (int64_t row = r0; row < r1; ++row) {
        const int64_t e0 = lp[row], e1 = lp[row + 1];
        double q[CPL];
#pragma unroll
        for (int u = 0; u < CPL; ++u) q[u] = 0.0;
        for (int64_t e = e0; e < e1; ++e) {
            const int32_t col = li[e];
            const double w = lv[e];
            Vec<CPL> pv;
            pv.load(P + col * ld + c);
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                double prod = w * pv.v[u];
                q[u] = q[u] + prod;
            }
        }
        Vec<CPL> qw;
#pragma unroll
        for (int u = 0; u < CPL; ++u) qw.v[u] = q[u];
        if (CPL == 1 || (live[0] && live[CPL - 1])) {
            qw.store(Q + row * ld + c);
        } else {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
                if (live[u]) Q[row * ld + c + u] = q[u];
        }
    }
}

// after the loop: the x update of the last executed iteration
__global__ void k_x_flush(CgGeom G, const double *__restrict__ P, const double *__restrict__ alpha,
                          const int32_t *__restrict__ xstep, int32_t it_last,
                          double *__restrict__ X) {
    int64_t ncol = G.col1 - G.col0;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < G.n * ncol;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = idx / ncol, c = G.col0 + idx % ncol;
        if (xstep[c] != it_last) continue;
        int64_t o = i * G.ld + c;
        double t1 = alpha[c] * P[o];
        X[o] = X[o] + t1;
    }
}

// plain dot accumulation (||b||^2 before the first iteration)
template <int CPL, int RU>
__global__ void __launch_bounds__(256) k_dot_acc(CgGeom G, ChunkArg ch,
                                                 const double *__restrict__ A,
                                                 const double *__restrict__ B,
                                                 double *__restrict__ acc) {
    const CgLane ln = cg_lane<CPL>(G);
    // lanes past the block's last column load nothing (their columns may lie
    // beyond the padded row, and past the buffer on the last row)
    if (!ln.ok || ln.c >= G.col1) return;
    const int64_t ld = G.ld, c = ln.c;
    const int64_t a = ch.a[ln.t], L = ch.len[ln.t];
    const int64_t n1 = L & ~(int64_t)15, n32 = n1 & ~(int64_t)31;
    double s[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) s[u] = 0.0;
    // RU chain rows per trip, loads first (absent rows re-read the first row)
    for (int64_t base = a + ln.j; base < a + n32; base += 32 * RU) {
        Vec<CPL> av[RU], bv[RU];
        bool ok[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
            ok[i] = base + 32 * i < a + n32;
            const int64_t row = ok[i] ? base + 32 * i : base;
            av[i].load(A + row * ld + c);
            bv[i].load(B + row * ld + c);
        }
#pragma unroll
        for (int i = 0; i < RU; ++i)
#pragma unroll
            for (int u = 0; u < CPL; ++u) {
                const double f = __builtin_fma(av[i].v[u], bv[i].v[u], s[u]);
                s[u] = ok[i] ? f : s[u];
            }
    }
#pragma unroll
    for (int u = 0; u < CPL; ++u)
        if (c + u < G.col1) acc[((c + u - G.col0) * kMaxChunks + ln.t) * 32 + ln.j] = s[u];
}

// OpenBLAS ddot finish (see oracle_ddot), one wave per column, one lane per
// BLAS chunk t: fold of the chunk's 32 chains, its optional 16-row block and
// FMA tail, then the chunk dots added in order from 0.0 (a single chunk is
// returned as is).  Values of the (< 32) leftover rows of chunk t are A[row]
// and, when Bside != nullptr, Bside[(t*32 + row - a - n32) * ld] (else B[row]).
__device__ __forceinline__ double chunk_dot(const double *__restrict__ a32, int64_t a, int64_t L,
                                            int t, int64_t ld, int64_t c,
                                            const double *__restrict__ A,
                                            const double *__restrict__ B,
                                            const double *__restrict__ Bside) {
    const int64_t n1 = L & ~(int64_t)15, n32 = n1 & ~(int64_t)31;
    auto bval = [&](int64_t row) {
        return Bside ? Bside[((int64_t)t * 32 + (row - a - n32)) * ld + c] : B[row * ld + c];
    };
    double dot = 0.0;
    if (n1) {
        double b[16];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int l = 0; l < 4; ++l) b[4 * q + l] = a32[8 * q + l] + a32[8 * q + 4 + l];
        if (n1 > n32) {
#pragma unroll
            for (int jj = 0; jj < 16; ++jj) {
                const int64_t row = a + n32 + jj;
                b[jj] = __builtin_fma(A[row * ld + c], bval(row), b[jj]);
            }
        }
        double c4[4];
#pragma unroll
        for (int l = 0; l < 4; ++l) c4[l] = ((b[l] + b[4 + l]) + b[8 + l]) + b[12 + l];
        dot = (c4[0] + c4[2]) + (c4[1] + c4[3]);
    }
    double tv[15], ta[15];  // tail loads first, then the dependent FMA chain
#pragma unroll
    for (int i = 0; i < 15; ++i) {
        const int64_t row = a + n1 + i;
        const bool in = row < a + L;
        tv[i] = in ? bval(row) : 0.0;
        ta[i] = in ? A[row * ld + c] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 15; ++i)
        if (n1 + i < L) dot = __builtin_fma(tv[i], ta[i], dot);
    return dot;
}

// value of column c's dot product; call with the whole wave (lane = chunk)
__device__ __forceinline__ double ddot_finish_impl(const double *__restrict__ acc_c,
                                                   const int64_t *__restrict__ ca,
                                                   const int64_t *__restrict__ cl, int count,
                                                   int64_t ld, int64_t c,
                                                   const double *__restrict__ A,
                                                   const double *__restrict__ B,
                                                   const double *__restrict__ Bside) {
    const int lane = threadIdx.x & 63;
    double d = 0.0;
    if (lane < count) d = chunk_dot(acc_c + lane * 32, ca[lane], cl[lane], lane, ld, c, A, B, Bside);
    if (count == 1) return __shfl(d, 0);
    double total = 0.0;
    for (int t = 0; t < count; ++t) total = total + __shfl(d, t);
    return total;
}

__device__ __noinline__ double ddot_finish_wave(const double *__restrict__ acc_c,
                                                   const int64_t *__restrict__ ca,
                                                   const int64_t *__restrict__ cl, int count,
                                                   int64_t ld, int64_t c,
                                                   const double *__restrict__ A,
                                                   const double *__restrict__ B,
                                                   const double *__restrict__ Bside) {
    return ddot_finish_impl(acc_c, ca, cl, count, ld, c, A, B, Bside);
}

// one wave per column: c = col0 + blockIdx.x * waves + wave
__device__ __forceinline__ int64_t fin_column(const CgGeom &G) {
    return G.col0 + (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
}

// init: rho = b.b, bn = sqrt(rho), atol = rtol*bn; bn == 0 -> done (x = b)
__global__ void __launch_bounds__(256) k_fin_init(CgGeom G, const int64_t *__restrict__ ca,
                                                  const int64_t *__restrict__ cl, int count,
                                                  const double *__restrict__ acc,
                                                  const double *__restrict__ Rr, double rtol,
                                                  double *__restrict__ bn, double *__restrict__ atol,
                                                  double *__restrict__ rho,
                                                  int32_t *__restrict__ active,
                                                  int32_t *__restrict__ iters,
                                                  int32_t *__restrict__ xstep,
                                                  int32_t *__restrict__ nactive) {
    const int64_t c = fin_column(G);
    if (c >= G.col1) return;
    const double d = ddot_finish_wave(acc + (c - G.col0) * kMaxChunks * 32, ca, cl, count, G.ld, c,
                                      Rr, Rr, nullptr);
    if ((threadIdx.x & 63) != 0) return;
    double b = __builtin_sqrt(d);
    bn[c] = b;
    double at = rtol * b;  // max(atol=0, rtol*bnrm2)
    atol[c] = at;
    rho[c] = d;
    iters[c] = 0;
    xstep[c] = -2;
    int act = 1;
    if (b == 0.0) act = 0;                     // cg returns b, info 0
    else if (__builtin_sqrt(d) < at) act = 0;  // converged at loop top, iteration 0
    active[c] = act;
    if (act) atomicAdd(nactive, 1);
}

__global__ void __launch_bounds__(256) k_fin_pq(CgGeom G, const int64_t *__restrict__ ca,
                                                const int64_t *__restrict__ cl, int count,
                                                const double *__restrict__ acc,
                                                const double *__restrict__ P,
                                                const double *__restrict__ Qfull,
                                                const double *__restrict__ qside,
                                                const double *__restrict__ rho,
                                                const int32_t *__restrict__ active, int32_t it,
                                                double *__restrict__ alpha,
                                                int32_t *__restrict__ xstep) {
    const int64_t c = fin_column(G);
    if (c >= G.col1 || !active[c]) return;
    const double pq = ddot_finish_wave(acc + (c - G.col0) * kMaxChunks * 32, ca, cl, count, G.ld,
                                       c, P, Qfull, qside);
    if ((threadIdx.x & 63) != 0) return;
    alpha[c] = rho[c] / pq;
    xstep[c] = it;  // x += alpha p is applied by the next k_cg_pq (or the flush)
}

// after the update of iteration `it`: rho_prev = rho; rho = r.r; loop-top test
__global__ void __launch_bounds__(256) k_fin_rr(CgGeom G, const int64_t *__restrict__ ca,
                                                const int64_t *__restrict__ cl, int count,
                                                const double *__restrict__ acc,
                                                const double *__restrict__ Rr, int32_t it,
                                                double *__restrict__ rho,
                                                double *__restrict__ rho_prev,
                                                const double *__restrict__ atol,
                                                int32_t *__restrict__ active,
                                                int32_t *__restrict__ iters,
                                                int32_t *__restrict__ nactive) {
    const int64_t c = fin_column(G);
    if (c >= G.col1 || !active[c]) return;
    const double rr = ddot_finish_wave(acc + (c - G.col0) * kMaxChunks * 32, ca, cl, count, G.ld,
                                       c, Rr, Rr, nullptr);
    if ((threadIdx.x & 63) != 0) return;
    rho_prev[c] = rho[c];
    rho[c] = rr;
    iters[c] = it + 1;
    if (__builtin_sqrt(rr) < atol[c]) {
        active[c] = 0;
        atomicSub(nactive, 1);
    }
}

// x = b for columns with ||b|| == 0 (cg returns b); zero X elsewhere
__global__ void k_x_init(CgGeom G, const double *__restrict__ Rr, const double *__restrict__ bn,
                         double *__restrict__ X) {
    int64_t ncol = G.col1 - G.col0;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < G.n * ncol;
         idx += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = idx / ncol, c = G.col0 + idx % ncol;
        int64_t o = i * G.ld + c;
        X[o] = (bn[c] == 0.0) ? Rr[o] : 0.0;
    }
}

// ---------------------------------------------------------------- scores
// r_eff[e] = 0 + pw_sum_c (Z_u,c - Z_v,c)^2 over columns [col0,col1),
// Z = nan_to_num(X) (metrics.py:288,292-293); finalize: :296-297.
__global__ void k_er_scores(const int32_t *__restrict__ rows, const int32_t *__restrict__ ix,
                            const double *__restrict__ X, int64_t ld, int64_t col0, int64_t col1,
                            int64_t e0, int64_t e1, int finalize, double *__restrict__ out) {
    for (int64_t e = e0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < e1;
         e += (int64_t)gridDim.x * blockDim.x) {
        const double *zu = X + (int64_t)rows[e] * ld + col0;
        const double *zv = X + (int64_t)ix[e] * ld + col0;
        double s = pw_sum<double>(col1 - col0, [&](int64_t c) {
            double a = zu[c], b = zv[c];
            if (a != a || __builtin_isinf(a)) a = 0.0;
            if (b != b || __builtin_isinf(b)) b = 0.0;
            double d = a - b;
            return d * d;
        });
        if (finalize) {
            s = 0.0 + s;
            if (s != s || __builtin_isinf(s)) s = 1e-10;
            s = s > 1e-10 ? s : 1e-10;
        }
        out[e - e0] = s;
    }
}

// ---------------------------------------------------------------- resident CG (mode 4)
// One workgroup (1024 threads, one per CU) owns whole columns: every iteration
// of a column's solve runs inside one launch, the dot products are workgroup
// reductions (no grid-wide step, no per-iteration launches), and the column's
// vectors live in column-major slots -- r, p, q per workgroup (reused from
// column to column) and x in its column of Xc.  256 resident columns x 4
// vectors fit the 256 MiB Infinity Cache for n up to ~24K, so the CG streams
// are served on-die rather than from HBM.  Per iteration:
//   p   (row-flat)  x += fl(alpha_{t-1} p_{t-1}); p = fl(fl(beta p) + r)
//   q   (row-flat)  q = L_reg p from a SELL-16 copy of L_reg (coalesced index
//                   loads, all gathers of a trip in flight), stored
//   pq  (chains)    thread `chain` = (BLAS chunk t, residue j) folds
//                   fma(p_i, q_i) over rows a_t + j, +32, ... -- the OpenBLAS
//                   accumulator chain -- then wave 0 finishes (ddot_finish_wave)
//   r   (chains)    r -= fl(alpha q), chains of dot(r, r), finish
static constexpr int kResThreads = 1024;
static constexpr int kResWaves = kResThreads / 64;
static constexpr int kSell = 16;  // SELL slice height: rows per block (padding to the block's longest row)

struct ResArgs {
    int64_t n, ld, ldn, col0, ncols;
    const int64_t *lp;
    const int32_t *li;
    const double *lv;
    const double *Rr;        // b = Y, row-major (stride ld)
    double *Xc;              // x, column-major: column col0 + i at Xc + i * ldn
    double *slots;           // per workgroup r, p, q (ldn each)
    const int64_t *ca, *cl;  // chunk starts / lengths (device, read by the finish)
    int32_t maxiter;
    double rtol;
    int32_t *iters;          // [k] iterations executed per column
    // SELL-16 copy of L_reg: block b = rows 16 b + l (l < 16); entry k of
    // row 16 b + l at soff[b] + 16 k + l
    const int64_t *soff;     // entry offset of each block
    const int32_t *swid;     // width (longest row) of each block
    const int32_t *scol;     // column, -1 = padding
    const double *sval;      // weight (nullptr in the unit-weight form)
    const double *sdiag;     // unit-weight form: L_reg_ii (off-diagonal entries are -1.0)
    // ELL copy of L_reg when every row has <= 16 entries: entry k of row i at
    // ecol[k * lde + i] (column-major, so a wave's loads are contiguous)
    const int32_t *ecol;     // column, -1 = padding
    const double *eval;      // weight (nullptr in the unit-weight form)
    int64_t lde;
    int64_t ql;              // rows of q mirrored in LDS (dynamic shared memory)
    int64_t nstab;           // SELL slices whose (offset, width) are staged in LDS after q (0: none)
    long long *prof;         // optional: workgroup 0's phase times (wall clock ticks)
    int32_t dcount;          // unit form: every L_reg_ii == fl((entries of row i) - 1 + 1e-6)
};

// a wave-uniform copy of v (read from lane 0): loop and branch conditions that
// depend on it compile as scalar branches, so every barrier stays in uniform
// control flow
__device__ __forceinline__ double wave_uniform(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// q = L_reg p over all rows, row-flat: wave w takes SELL blocks w, w + 16, ...,
// RB blocks per trip; fold from 0.0 in ascending column with rounded products
// (SciPy csr_matvec).  The first W entries of each row are loaded at once
// (then all their gathers), wider rows finish in a tail loop.
template <int RB, int W, bool UNIT>
__device__ __forceinline__ void res_spmv(const ResArgs &A, const double *p, double *q, double *sq, int64_t ql,
                                         const int2 *stab) {
    const int64_t n = A.n;
    const int64_t ntile = (n + 63) >> 6;  // 64-row tiles, one per wave-trip row
    for (int64_t t0 = threadIdx.x >> 6; t0 < ntile; t0 += (int64_t)kResWaves * RB) {
        int64_t o[RB], row[RB];
        int32_t w[RB], wmax = 0;
        double acc[RB], dg[RB];
        bool ok[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int64_t t = t0 + (int64_t)kResWaves * i;
            const int64_t rw = (t < ntile ? t : t0) * 64 + (threadIdx.x & 63);
            ok[i] = t < ntile && rw < n;
            row[i] = ok[i] ? rw : 0;
            const int64_t b = row[i] / kSell;
            int32_t wb;
            if (stab) {  // slice table staged in LDS: no dependent global load
                const int2 t = stab[b];
                o[i] = (int64_t)t.x + row[i] % kSell;
                wb = t.y;
            } else {
                o[i] = A.soff[b] + row[i] % kSell;
                wb = A.swid[b];
            }
            w[i] = ok[i] ? wb : 0;
            wmax = w[i] > wmax ? w[i] : wmax;
            // the diagonal: derived from the row's entry count when the whole row is in
            // the first W entries (dcount graphs), else loaded
            dg[i] = (UNIT && !(A.dcount && w[i] <= W)) ? A.sdiag[row[i]] : 0.0;
            acc[i] = 0.0;
        }
        {
            int32_t col[RB][W];
            double v[RB][W], pv[RB][W];
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int k = 0; k < W; ++k) {
                    const int64_t idx = o[i] + (k < w[i] ? kSell * k : 0);
                    col[i][k] = A.scol[idx];
                    if (!UNIT) v[i][k] = A.sval[idx];
                }
            if (UNIT && A.dcount) {
#pragma unroll
                for (int i = 0; i < RB; ++i)
                    if (w[i] <= W) {
                        int cnt = 0;
#pragma unroll
                        for (int k = 0; k < W; ++k) cnt += (k < w[i] && col[i][k] >= 0) ? 1 : 0;
                        dg[i] = (double)(cnt - 1) + 1e-6;
                    }
            }
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int k = 0; k < W; ++k) pv[i][k] = p[col[i][k] >= 0 ? col[i][k] : 0];
#pragma unroll
            for (int i = 0; i < RB; ++i)
#pragma unroll
                for (int k = 0; k < W; ++k) {
                    if (UNIT) v[i][k] = col[i][k] == row[i] ? dg[i] : -1.0;
                    const double prod = v[i][k] * pv[i][k];
                    const double qn = acc[i] + prod;
                    acc[i] = (k < w[i] && col[i][k] >= 0) ? qn : acc[i];
                }
        }
        for (int32_t k = W; k < wmax; ++k) {
            int32_t col[RB];
            double v[RB], pv[RB];
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                const int64_t idx = o[i] + (k < w[i] ? (int64_t)kSell * k : 0);
                col[i] = A.scol[idx];
                v[i] = UNIT ? 0.0 : A.sval[idx];
            }
#pragma unroll
            for (int i = 0; i < RB; ++i) pv[i] = p[col[i] >= 0 ? col[i] : 0];
#pragma unroll
            for (int i = 0; i < RB; ++i) {
                if (UNIT) v[i] = col[i] == row[i] ? dg[i] : -1.0;
                const double prod = v[i] * pv[i];
                const double qn = acc[i] + prod;
                acc[i] = (k < w[i] && col[i] >= 0) ? qn : acc[i];
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i)
            if (ok[i]) {  // rows mirrored in LDS live only there (chunk tails: copied below)
                if (row[i] < ql) sq[row[i]] = acc[i];
                else q[row[i]] = acc[i];
            }
    }
}

// q = L_reg p over all rows from the ELL copy: row-flat, RB rows per thread
// and trip, all W index loads, then all W gathers of each row in flight (two
// dependent memory latencies per trip); padding entries are masked.
template <int RB, int W, bool UNIT>
__device__ __forceinline__ void res_spmv_ell(const ResArgs &A, const double *p, double *q, double *sq, int64_t ql) {
    const int64_t n = A.n;
    for (int64_t r0 = threadIdx.x; r0 < n; r0 += (int64_t)kResThreads * RB) {
        int64_t row[RB];
        bool ok[RB];
        int32_t col[RB][W];
        double v[RB][W], pv[RB][W], dg[RB];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            const int64_t rw = r0 + (int64_t)kResThreads * i;
            ok[i] = rw < n;
            row[i] = ok[i] ? rw : r0;
            dg[i] = UNIT ? A.sdiag[row[i]] : 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                col[i][k] = A.ecol[k * A.lde + row[i]];
                if (!UNIT) v[i][k] = A.eval[k * A.lde + row[i]];
            }
        }
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
            for (int k = 0; k < W; ++k) pv[i][k] = p[col[i][k] >= 0 ? col[i][k] : 0];
#pragma unroll
        for (int i = 0; i < RB; ++i) {
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                if (UNIT) v[i][k] = col[i][k] == row[i] ? dg[i] : -1.0;
                const double prod = v[i][k] * pv[i][k];
                const double qn = acc + prod;
                acc = col[i][k] >= 0 ? qn : acc;
            }
            if (ok[i]) {
                if (row[i] < ql) sq[row[i]] = acc;
                else q[row[i]] = acc;
            }
        }
    }
}

template <int RB, int W, int RC, bool UNIT, int EW>
__global__ void __launch_bounds__(kResThreads) k_cg_resident(ResArgs A, ChunkArg ch) {
    __shared__ double s_acc[kMaxChunks * 32];
    __shared__ double s_bc;
    extern __shared__ double sq[];  // q of rows < ql (LDS mirror of the q slot), then the slice table
    const int tid = threadIdx.x;
    const int nchains = ch.count * 32;
    const int64_t n = A.n, ql = A.ql;
    int2 *stab = reinterpret_cast<int2 *>(sq + ql);
    for (int64_t b = tid; b < A.nstab; b += kResThreads)
        stab[b] = make_int2((int)A.soff[b], A.swid[b]);
    __syncthreads();
    double *r = A.slots + (int64_t)blockIdx.x * 3 * A.ldn;
    double *p = r + A.ldn;
    double *q = p + A.ldn;

    // phase clock (workgroup 0, thread 0 writes it out at the end): p update,
    // SpMV, pq chains, r update, finish (incl. the barrier wait before it)
    long long tp[5] = {0, 0, 0, 0, 0};
    long long tmark = wall_clock64();
    auto lap = [&](int ph) {
        const long long t = wall_clock64();
        tp[ph] += t - tmark;
        tmark = t;
    };
    // chain partials are in s_acc: wave 0 finishes in OpenBLAS order, all read it
    auto finish = [&](const double *X, const double *Y) -> double {
        __syncthreads();
        if (tid < 64) {
            const double d = ddot_finish_impl(s_acc, A.ca, A.cl, ch.count, 1, 0, X, Y, nullptr);
            if (tid == 0) s_bc = d;
        }
        __syncthreads();
        lap(4);
        return wave_uniform(s_bc);
    };
    // chain (t, j): rows a_t + j + 32 s below e32 = a_t + (len_t rounded down to 32 after 16)
    auto chain_geom = [&](int chain, int64_t &a, int64_t &L, int64_t &e32) {
        const int t = chain >> 5;
        a = ch.a[t] + (chain & 31);
        L = ch.a[t] + ch.len[t];
        e32 = ch.a[t] + ((ch.len[t] & ~(int64_t)15) & ~(int64_t)31);
    };
    // fold fma(X_i, Y_i) along every chain into s_acc (loads of RC rows in flight);
    // YQ: Y is q, read from its LDS mirror where it has one
    auto chain_dot = [&](const double *X, const double *Y, bool YQ) {
        for (int chain = tid; chain < nchains; chain += kResThreads) {
            int64_t a, L, e32;
            chain_geom(chain, a, L, e32);
            double s = 0.0;
            for (int64_t base = a; base < e32; base += 32 * RC) {
                double xv[RC], yv[RC];
#pragma unroll
                for (int i = 0; i < RC; ++i) {
                    const int64_t rw = base + 32 * i < e32 ? base + 32 * i : base;
                    xv[i] = X[rw];
                    yv[i] = (YQ && rw < ql) ? sq[rw] : Y[rw];
                }
#pragma unroll
                for (int i = 0; i < RC; ++i)
                    if (base + 32 * i < e32) s = __builtin_fma(xv[i], yv[i], s);
            }
            s_acc[chain] = s;
        }
    };

    // columns dealt round-robin; every loop and branch below is workgroup-uniform
    for (int64_t ci = blockIdx.x; ci < A.ncols; ci += gridDim.x) {
        const int64_t c = A.col0 + ci;
        double *x = A.Xc + ci * A.ldn;
        for (int64_t i = tid; i < n; i += kResThreads) r[i] = A.Rr[i * A.ld + c];
        __syncthreads();
        chain_dot(r, r, false);  // ||b||^2 = rho_0 (r = b.copy())
        double rr = finish(r, r);
        const double bn = __builtin_sqrt(rr);
        const double atol = A.rtol * bn;  // max(atol=0, rtol*bnrm2)
        int32_t done = 0;
        double rho_prev = 0.0, alpha_prev = 0.0;
        const bool act = !(bn == 0.0) && !(__builtin_sqrt(rr) < atol);
        for (int32_t it = 0; act && it < A.maxiter; ++it) {
            if (it > 0 && __builtin_sqrt(rr) < atol) break;  // loop-top test
            const double rho_cur = rr;
            const double beta = it > 0 ? rho_cur / rho_prev : 0.0;
            lap(4);
            // p = beta p + r (two roundings); the x update of iteration it-1 rides along
            if (it == 0) {
                for (int64_t i = tid; i < n; i += kResThreads) p[i] = r[i];
            } else {
                // 8 rows per thread in flight as 4 row pairs (16-B loads; the odd row n of
                // an odd n is slot padding, written but never read)
                constexpr int U = 6;
                const int64_t n2 = (n + 1) >> 1;
                double2 *p2 = reinterpret_cast<double2 *>(p);
                const double2 *r2 = reinterpret_cast<const double2 *>(r);
                double2 *x2 = reinterpret_cast<double2 *>(x);
                for (int64_t j0 = tid; j0 < n2; j0 += kResThreads * U) {
                    double2 po[U], rv[U], xv[U];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int64_t j = j0 + (int64_t)u * kResThreads;
                        const int64_t jc = j < n2 ? j : j0;
                        po[u] = p2[jc];
                        rv[u] = r2[jc];
                        xv[u] = it > 1 ? x2[jc] : make_double2(0.0, 0.0);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int64_t j = j0 + (int64_t)u * kResThreads;
                        if (j < n2) {
                            double2 xo, pn;
                            const double t1a = alpha_prev * po[u].x, t1b = alpha_prev * po[u].y;
                            xo.x = xv[u].x + t1a;
                            xo.y = xv[u].y + t1b;
                            const double pba = po[u].x * beta, pbb = po[u].y * beta;
                            pn.x = pba + rv[u].x;
                            pn.y = pbb + rv[u].y;
                            x2[j] = xo;
                            p2[j] = pn;
                        }
                    }
                }
            }
            __syncthreads();
            lap(0);
            if (EW) res_spmv_ell<EW <= 8 ? 2 : 1, EW, UNIT>(A, p, q, sq, ql);
            else res_spmv<RB, W, UNIT>(A, p, q, sq, ql, A.nstab ? stab : nullptr);
            __syncthreads();
            lap(1);
            chain_dot(p, q, true);
            // the chunk tails (< 32 rows past each chunk's chains) are read from the q slot
            // by the finish and the r update: copy the LDS-only ones there
            for (int k = tid; k < nchains; k += kResThreads) {
                int64_t a, L, e32;
                chain_geom(k, a, L, e32);
                const int64_t rw = e32 + (k & 31);
                if (rw < L && rw < ql) q[rw] = sq[rw];
            }
            lap(2);
            const double pq = finish(p, q);
            const double alpha = rho_cur / pq;
            // r -= alpha q, chains of dot(r, r); the < 32 leftover rows of each chunk too
            for (int chain = tid; chain < nchains; chain += kResThreads) {
                int64_t a, L, e32;
                chain_geom(chain, a, L, e32);
                double s = 0.0;
                for (int64_t base = a; base < e32; base += 32 * RC) {
                    double rv[RC], qv[RC];
#pragma unroll
                    for (int i = 0; i < RC; ++i) {
                        const int64_t rw = base + 32 * i < e32 ? base + 32 * i : base;
                        rv[i] = r[rw];
                        qv[i] = rw < ql ? sq[rw] : q[rw];
                    }
#pragma unroll
                    for (int i = 0; i < RC; ++i)
                        if (base + 32 * i < e32) {
                            const double t2 = alpha * qv[i];
                            const double rn = rv[i] - t2;
                            r[base + 32 * i] = rn;
                            s = __builtin_fma(rn, rn, s);
                        }
                }
                const int64_t lr = e32 + (chain & 31);
                if (lr < L) {
                    const double t2 = alpha * q[lr];
                    r[lr] = r[lr] - t2;
                }
                s_acc[chain] = s;
            }
            lap(3);
            rr = finish(r, r);
            rho_prev = rho_cur;
            alpha_prev = alpha;
            done = it + 1;
        }
        // x: b (||b|| == 0), 0 (no iteration), or the last pending update
        if (bn == 0.0) {
            for (int64_t i = tid; i < n; i += kResThreads) x[i] = r[i];
        } else if (done == 0) {
            for (int64_t i = tid; i < n; i += kResThreads) x[i] = 0.0;
        } else {
            for (int64_t i = tid; i < n; i += kResThreads) {
                const double t1 = alpha_prev * p[i];
                x[i] = (done > 1 ? x[i] : 0.0) + t1;
            }
        }
        if (tid == 0) A.iters[c] = done;
    }
    if (A.prof && blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < 5; ++i) A.prof[i] = tp[i];
}

// unit-weight test: every off-diagonal entry of L_reg is -1.0 (clears *flag otherwise);
// diag[i] = L_reg_ii (0.0 where the diagonal entry was dropped)
__global__ void k_l_unit(const int64_t *__restrict__ lp, const int32_t *__restrict__ li,
                         const double *__restrict__ lv, int64_t n, double *__restrict__ diag,
                         int32_t *__restrict__ flag) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        double dg = 0.0;
        bool unit = true;
        for (int64_t e = lp[i]; e < lp[i + 1]; ++e) {
            if (li[e] == i) dg = lv[e];
            else unit = unit && lv[e] == -1.0;
        }
        diag[i] = dg;
        if (!unit) atomicAnd(flag, ~1);
        if (!(dg == (double)(lp[i + 1] - lp[i] - 1) + 1e-6)) atomicAnd(flag, ~2);
    }
}

// ELL build (rows of at most lde-independent width W): one thread per row
__global__ void k_ell_fill(int64_t n, int W, int64_t lde, const int64_t *__restrict__ lp,
                           const int32_t *__restrict__ li, const double *__restrict__ lv,
                           int32_t *__restrict__ ecol, double *__restrict__ eval) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = lp[i], len = lp[i + 1] - e0;
        for (int k = 0; k < W; ++k) {
            ecol[k * lde + i] = k < len ? li[e0 + k] : -1;
            if (eval) eval[k * lde + i] = k < len ? lv[e0 + k] : 0.0;
        }
    }
}

// SELL-16 build: one thread per block (width), one per row (fill)
__global__ void k_sell_width(int64_t n, const int64_t *__restrict__ lp, int32_t *__restrict__ swid,
                             int64_t *__restrict__ cnt) {
    const int64_t nb = (n + kSell - 1) / kSell;
    for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nb;
         b += (int64_t)gridDim.x * blockDim.x) {
        int64_t w = 0;
        for (int64_t r = b * kSell; r < (b + 1) * kSell && r < n; ++r) {
            const int64_t l = lp[r + 1] - lp[r];
            w = l > w ? l : w;
        }
        swid[b] = (int32_t)w;
        cnt[b] = kSell * w;
    }
}

__global__ void k_sell_fill(int64_t n, const int64_t *__restrict__ lp,
                            const int32_t *__restrict__ li, const double *__restrict__ lv,
                            const int64_t *__restrict__ soff, const int32_t *__restrict__ swid,
                            int32_t *__restrict__ scol, double *__restrict__ sval) {
    for (int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; g < n;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = g / kSell;
        const int l = (int)(g % kSell);
        const int64_t e0 = lp[g], len = lp[g + 1] - e0;
        for (int64_t k = 0; k < swid[b]; ++k) {
            const int64_t idx = soff[b] + kSell * k + l;
            scol[idx] = k < len ? li[e0 + k] : -1;
            if (sval) sval[idx] = k < len ? lv[e0 + k] : 0.0;
        }
    }
}

// Xc (column-major, ncols x ldn) -> X (row-major, stride ld) columns [col0, col0+ncols)
__global__ void __launch_bounds__(256) k_cols_to_rows(const double *__restrict__ Xc, int64_t ldn,
                                                      int64_t n, int64_t col0, int64_t ncols,
                                                      double *__restrict__ X, int64_t ld) {
    __shared__ double tile[32][33];
    const int64_t r0 = (int64_t)blockIdx.x * 32, c0 = (int64_t)blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int yy = ty; yy < 32; yy += 8) {
        const int64_t col = c0 + yy, row = r0 + tx;
        if (col < ncols && row < n) tile[yy][tx] = Xc[col * ldn + row];
    }
    __syncthreads();
    for (int yy = ty; yy < 32; yy += 8) {
        const int64_t row = r0 + yy, col = c0 + tx;
        if (col < ncols && row < n) X[row * ld + col0 + col] = tile[tx][yy];
    }
}

static ChunkArg to_arg(const Chunks &c) {
    ChunkArg a{};
    a.count = c.count;
    for (int i = 0; i < c.count; ++i) {
        a.a[i] = c.a[i];
        a.len[i] = c.len[i];
    }
    return a;
}

}  // namespace gs

namespace gs {
// out = sum of v[0..n) (one workgroup; profiling bookkeeping)
__global__ void __launch_bounds__(256) k_sum_i32(const int32_t *__restrict__ v, int64_t n,
                                                 int64_t *__restrict__ out) {
    __shared__ int64_t part[256];
    int64_t acc = 0;
    for (int64_t i = threadIdx.x; i < n; i += 256) acc += v[i];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = part[0];
}

// Y[:, col0:col1] (+)= B @ (raw rows [e0, e1) / sqrt_k): raw is device-resident,
// row-major with kraw columns -- the whole NumPy rows (kraw = k) or just the slice
// (kraw = col1 - col0).  Advances the streamed-row cursor.
void project_rows(gs_ctx *c, int64_t e0, int64_t e1, const double *draw, int64_t kraw,
                  int64_t col0, int64_t col1, double sqrt_k) {
    ErState &er = c->er;
    const int64_t kc = col1 - col0, rc0 = kraw == er.k ? 0 : col0;
    const int64_t ncb = (kc + 63) / 64;
    hipEvent_t t0 = prof_begin(c);
    k_project<<<grid_for(er.n * ncb * 64, 256, 65536), 256, 0, c->stream>>>(
        er.bptr.as<int64_t>(), er.bcol.as<int64_t>(), er.bsgn.as<int8_t>(), er.n, col0, col1, kraw,
        rc0, er.ld, e0, e1, draw, sqrt_k, er.Rr.as<double>());
    GS_HIP(hipGetLastError());
    prof_end(c, t0, "er_project", 8.0 * (double)(e1 - e0) * (double)kc * 3.0);
    er.proj_c0 = col0;
    er.proj_c1 = col1;
    er.proj_next = e1;
}
}  // namespace gs

using namespace gs;

// every column of [c0, c1) solved since the last gs_er_prepare (a read of
// columns another rank -- or no one -- solved must not return stale X)
static bool er_cols_solved(const ErState &er, int64_t c0, int64_t c1) {
    if ((int64_t)er.col_solved.size() < c1) return false;
    for (int64_t i = c0; i < c1; ++i)
        if (!er.col_solved[i]) return false;
    return true;
}

extern "C" {

int gs_er_prepare(gs_ctx *c, int64_t k, double reg, int64_t *m_out) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        GS_CHECK(k >= 1, GS_EINVAL, "k must be >= 1");
        GS_HIP(hipSetDevice(c->device));
        ensure_transpose(c);
        Graph &g = c->g;
        ErState &er = c->er;
        int64_t n = g.n, nnz = g.nnz;
        er.proj_next = 0;
        er.solved = false;
        er.proj_c0 = 0;
        er.proj_c1 = k;
        // the edge ids, B and L_reg are functions of (graph, k, reg) only: a repeated
        // prepare (every bench step, every rank) reuses them -- no kernels, no host sync
        int64_t regbits;
        memcpy(&regbits, &reg, sizeof(regbits));
        const std::vector<int64_t> pkey = {g.epoch, k, regbits};
        er.col_solved.assign((size_t)k, 0);
        if (pkey == er.prep_key) {
            // per-column scalars and iteration counts restart (async, no host sync): a
            // column not solved since this prepare reports 0 iterations, as before
            GS_HIP(hipMemsetAsync(er.colstate.ptr, 0, er.colstate.bytes, c->stream));
            GS_HIP(hipMemsetAsync(er.iters.ptr, 0, sizeof(int32_t) * k, c->stream));
            if (m_out) *m_out = er.m;
            return;
        }
        er.prep_key.clear();
        er.n = n;
        er.k = k;
        er.reg = reg;
        // undirected edge ids (u<v in CSR order, metrics.py:236-242)
        int64_t *eid = (int64_t *)er.edge_id.ensure(sizeof(int64_t) * (nnz ? nnz : 1));
        int64_t m = 0;
        if (nnz) {
            int64_t *flag = (int64_t *)c->scratch[0].ensure(sizeof(int64_t) * nnz);
            int64_t *pos = (int64_t *)c->scratch[1].ensure(sizeof(int64_t) * nnz);
            k_upper_flags<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(
                g.rows.as<int32_t>(), g.indices.as<int32_t>(), nnz, flag);
            exclusive_scan_i64(c, flag, pos, nnz);
            k_edge_ids<<<grid_for(nnz, 256, 8192), 256, 0, c->stream>>>(flag, pos, nnz, eid);
            int64_t last[2];
            GS_HIP(hipMemcpyAsync(&last[0], pos + nnz - 1, 8, hipMemcpyDeviceToHost, c->stream));
            GS_HIP(hipMemcpyAsync(&last[1], flag + nnz - 1, 8, hipMemcpyDeviceToHost, c->stream));
            GS_HIP(hipStreamSynchronize(c->stream));
            m = last[0] + last[1];
        }
        er.m = m;
        // incidence rows B (metrics.py:260-269)
        int64_t *cnt = (int64_t *)c->scratch[0].ensure(sizeof(int64_t) * (n + 1));
        GS_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (n + 1), c->stream));
        int64_t *bptr = (int64_t *)er.bptr.ensure(sizeof(int64_t) * (n + 1));
        if (n)
            k_b_counts<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(
                g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.tptr.as<int64_t>(),
                g.tidx.as<int32_t>(), n, cnt);
        exclusive_scan_i64(c, cnt, bptr, n + 1);
        er.bcol.ensure(sizeof(int64_t) * (2 * m + 1));
        er.bsgn.ensure(2 * m + 1);
        er.bcur.ensure(sizeof(int64_t) * (n + 1));
        if (n)
            k_b_fill<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(
                g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.tptr.as<int64_t>(),
                g.tidx.as<int32_t>(), g.tpos.as<int64_t>(), eid, n, bptr, er.bcol.as<int64_t>(),
                er.bsgn.as<int8_t>(), er.bcur.as<int64_t>());
        // L_reg (metrics.py:251-256)
        GS_HIP(hipMemsetAsync(cnt, 0, sizeof(int64_t) * (n + 1), c->stream));
        int64_t *lp = (int64_t *)er.lp.ensure(sizeof(int64_t) * (n + 1));
        if (n)
            k_l_counts<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(
                g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.data.as<double>(), n, reg, cnt);
        exclusive_scan_i64(c, cnt, lp, n + 1);
        int64_t lnnz = 0;
        GS_HIP(hipMemcpyAsync(&lnnz, lp + n, 8, hipMemcpyDeviceToHost, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        er.lnnz = lnnz;
        er.li.ensure(sizeof(int32_t) * (lnnz + 1));
        er.lv.ensure(sizeof(double) * (lnnz + 1));
        if (n)
            k_l_fill<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(
                g.indptr.as<int64_t>(), g.indices.as<int32_t>(), g.data.as<double>(), n, reg, lp,
                er.li.as<int32_t>(), er.lv.as<double>());
        // state
        // row stride padded to 8 doubles: 64-B aligned rows, 16-B vector access
        er.ld = (k + 7) & ~(int64_t)7;
        // + slack: a 16-B access of a block's last (odd) column reads one column past
        // the block, which on the last row may be past the row's padding
        size_t nk = sizeof(double) * ((size_t)(n ? n : 1) * (size_t)er.ld + 256);
        er.X.ensure(nk);
        er.Rr.ensure(nk);
        er.P0.ensure(nk);
        er.P1.ensure(nk);
        er.Q.ensure(nk);
        // the projection writes every Y entry it covers (the first rows fold from 0.0);
        // the row padding past k is zeroed once per allocation
        if (er.rr_zeroed != er.Rr.ptr || er.rr_k != k) {
            GS_HIP(hipMemsetAsync(er.Rr.ptr, 0, er.Rr.bytes, c->stream));
            er.rr_zeroed = er.Rr.ptr;
            er.rr_k = k;
        }
        er.colstate.ensure(sizeof(double) * 5 * k + sizeof(int32_t) * (3 * k + 4));
        GS_HIP(hipMemsetAsync(er.colstate.ptr, 0, er.colstate.bytes, c->stream));
        er.acc.ensure(sizeof(double) * (size_t)k * kMaxChunks * 32);
        er.iters.ensure(sizeof(int32_t) * k);
        GS_HIP(hipMemsetAsync(er.iters.ptr, 0, sizeof(int32_t) * k, c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        er.prep_key = pkey;
        if (m_out) *m_out = m;
    });
}

int gs_er_project_rows_cols(gs_ctx *c, int64_t e0, int64_t e1, const double *raw, int loc,
                            double sqrt_k, int64_t col0, int64_t col1) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.k > 0, GS_ESTATE, "gs_er_prepare first");
        GS_CHECK(e0 == er.proj_next && e0 <= e1 && e1 <= er.m, GS_EINVAL,
                 "rows must be streamed in order: expected %lld, got [%lld, %lld) of %lld",
                 (long long)er.proj_next, (long long)e0, (long long)e1, (long long)er.m);
        GS_CHECK(0 <= col0 && col0 < col1 && col1 <= er.k, GS_EINVAL, "bad column range");
        GS_CHECK(e0 == 0 || (col0 == er.proj_c0 && col1 == er.proj_c1), GS_EINVAL,
                 "every row chunk must project the same columns");
        GS_HIP(hipSetDevice(c->device));
        er.proj_c0 = col0;
        er.proj_c1 = col1;
        int64_t rowsn = e1 - e0;
        if (rowsn == 0) return;
        size_t bytes = sizeof(double) * (size_t)rowsn * (size_t)er.k;
        const double *draw = (const double *)to_device(c, er.rawbuf, raw, bytes, loc);
        project_rows(c, e0, e1, draw, er.k, col0, col1, sqrt_k);
        if (loc == GS_HOST) GS_HIP(hipStreamSynchronize(c->stream));  // rawbuf reuse
    });
}

int gs_er_project_rows(gs_ctx *c, int64_t e0, int64_t e1, const double *raw, int loc,
                       double sqrt_k) {
    const int64_t k = c ? c->er.k : 0;
    return gs_er_project_rows_cols(c, e0, e1, raw, loc, sqrt_k, 0, k > 0 ? k : 1);
}

int gs_er_solve(gs_ctx *c, int64_t col0, int64_t col1, int32_t maxiter, double rtol,
                int32_t blas_threads) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.k > 0, GS_ESTATE, "gs_er_prepare first");
        GS_CHECK(er.proj_next == er.m, GS_ESTATE, "projection incomplete: %lld of %lld rows",
                 (long long)er.proj_next, (long long)er.m);
        GS_CHECK(0 <= col0 && col0 < col1 && col1 <= er.k, GS_EINVAL, "bad column range");
        GS_CHECK(er.proj_c0 <= col0 && col1 <= er.proj_c1, GS_ESTATE,
                 "columns [%lld, %lld) were not projected (Y holds [%lld, %lld))", (long long)col0,
                 (long long)col1, (long long)er.proj_c0, (long long)er.proj_c1);
        GS_HIP(hipSetDevice(c->device));
        const int64_t n = er.n, k = er.k;
        // OpenBLAS caps its thread count at MAX_THREADS (64 in NumPy's build): a larger
        // request runs -- and orders the ddot sums -- as 64 threads
        if (blas_threads > kMaxChunks) blas_threads = kMaxChunks;
        ChunkArg ch = to_arg(make_chunks(n, blas_threads));
        // two columns per lane (16-B accesses) unless that leaves too few waves
        const int64_t ncols = col1 - col0;
        const int64_t waves2 = ((ncols + 127) / 128) * 32 * (int64_t)ch.count;
        int cpl = waves2 >= 4096 ? 2 : 1;
        if (const char *e = getenv("GSPARSE_CG_CPL")) cpl = atoi(e) == 1 ? 1 : 2;
        CgGeom G;
        G.n = n;
        G.k = k;
        G.ld = er.ld;
        G.col0 = col0;
        G.col1 = col1;
        G.ncb = (int32_t)((ncols + 64 * cpl - 1) / (64 * cpl));
        G.npairs = G.ncb * ch.count;
        ColPtrs cp = col_ptrs(er);
        double *X = er.X.as<double>(), *Rr = er.Rr.as<double>();
        // mode 0 (short rows, default): q recomputed in k_cg_upd from the stored p
        // (one gather per entry is cheaper than 16 B/entry more of stream); only
        // the q of the < 32 leftover rows per chunk is kept, for the finish.
        // 1: q stored by the fused p/q kernel (GSPARSE_CG_STOREQ=1 selects it);
        // 2: split p stream + SpMV on the stored p (long rows: one gather per entry
        // instead of the fused kernel's two); 3: as 2 with the SpMV in
        // column-block-major order (gathers served by the Infinity Cache) and a
        // separate dot(p,q) pass -- the default for long rows.  GSPARSE_CG_MODE overrides.
        // Short rows: recompute (0) while the chains give enough waves; fewer
        // columns (a rank's share on N GPUs) -> stored q (1), then the split
        // kernels (3); measured on Roman at k/1, k/2, k/4, k/8 columns.
        // Resident solver (4) where its 256 columns in flight fit the Infinity Cache
        // (4 vectors x 8 B x n x 256 <= ~200 MB) and the BLAS chunks give >= 128 chains:
        // Roman size, 2,674 columns: 0.51 s vs 0.53 s for mode 0; k/8 columns ~0.09 s vs 0.12 s.
        const bool resident = n > 10000 && n <= 24576 && ch.count >= 4 &&
                              er.lnnz <= kStoreQRowLen * n;
        // register-resident solver (5) where its 512-thread form applies (Roman size:
        // 55.7 vs 76.4 us per column-iteration for mode 4); its
        // 256-thread form (more rows per thread) is no faster than mode 4: opt-in
        const bool regres = cg_regres_applies(n, ch.count, ch.len);
        const bool regwide = cg_regres_wide(n, ch.count, ch.len);
        int mode = resident && regwide                        ? 5
                   : resident                                 ? 4
                   : (n > 0 && er.lnnz > kStoreQRowLen * n) ? 3
                   : ncols >= 2048                          ? 0
                   : ncols >= 512                           ? 1
                                                            : 3;
        if (const char *e = getenv("GSPARSE_CG_MODE")) {
            const int v = atoi(e);
            mode = (v >= 0 && v <= 5) ? v : 0;
            if (mode == 5 && !regres) mode = 4;
        }
        if (const char *e = getenv("GSPARSE_CG_STOREQ")) mode = atoi(e) != 0 ? 1 : 0;
        const bool storeq = mode != 0;
        // chain rows per trip in the fused kernels (loads of all of them in flight)
        // (fewer waves -> more rows per trip; measured on Roman at k/1 .. k/8 columns)
        const int64_t cg_waves = (int64_t)G.ncb * ch.count * 32;
        int ru = cg_waves >= 4096 ? 1 : cg_waves >= 2048 ? 2 : 4;
        if (const char *e = getenv("GSPARSE_CG_RU")) {
            const int v = atoi(e);
            ru = (v == 1 || v == 2 || v == 4 || v == 8) ? v : ru;
        }
        double *Qbuf = (double *)er.Q.ensure(
            storeq ? sizeof(double) * (size_t)n * (size_t)er.ld
                   : sizeof(double) * (size_t)ch.count * 32 * (size_t)er.ld);
        double *qside = storeq ? nullptr : Qbuf;
        double *Qfull = storeq ? Qbuf : nullptr;
        double *P[2] = {er.P0.as<double>(), er.P1.as<double>()};
        double *acc = er.acc.as<double>();
        // 8 workgroups (32 residues) per (column block, chunk) pair, XCD-grouped
        dim3 grid((unsigned)(((G.npairs + 7) / 8) * 64)), block(256);
        // finish kernels: one wave per column, one lane per BLAS chunk
        const unsigned fgrid = grid_for(ncols, 4);
        int64_t hch[2 * kMaxChunks];
        for (int t = 0; t < ch.count; ++t) {
            hch[t] = ch.a[t];
            hch[kMaxChunks + t] = ch.len[t];
        }
        auto *dch = (int64_t *)c->buf("er_chunks").ensure(sizeof(hch));
        GS_HIP(hipMemcpyAsync(dch, hch, sizeof(hch), hipMemcpyHostToDevice, c->stream));
        const int64_t *ca = dch, *cl = dch + kMaxChunks;
        // algorithmic bytes, SURVEY 8(d) B_ER: per column and iteration 8 (nnz(L_reg) + 10 n),
        // i.e. one 8-B p read per L_reg entry (the SpMV) + the vector streams.  Attributed
        // to the kernel that does each part: pq reads x, p, r and writes x, p (first
        // iteration: r in, p out) and performs the SpMV (+ q written when stored); upd
        // reads p (or q), r and writes r (its q recompute is not counted again)
        const double qb = storeq ? 8.0 : 0.0;
        const double lnz = (double)er.lnnz;
        const double bytes_pq = ((40.0 + qb) * n + 8.0 * lnz) * ncols,
                     bytes_pq0 = ((16.0 + qb) * n + 8.0 * lnz) * ncols,
                     bytes_upd = 24.0 * n * ncols;
        const int64_t *lp = er.lp.as<int64_t>();
        const int32_t *li = er.li.as<int32_t>();
        const double *lv = er.lv.as<double>();
        if (mode == 4 || mode == 5) {
            // resident solvers: one workgroup per CU, whole columns per workgroup
            const int64_t ldn = (n + 7) & ~(int64_t)7;
            int64_t slots = 256;
            if (const char *e = getenv("GSPARSE_CG_SLOTS")) slots = atoi(e) > 0 ? atoi(e) : slots;
            if (slots > ncols) slots = ncols;
            // as few workgroups as the round count allows (every workgroup then owns the
            // same number of columns, and fewer CUs share the Infinity Cache in each round)
            if (slots > 0 && !getenv("GSPARSE_CG_SLOTS")) {
                const int64_t rounds = (ncols + slots - 1) / slots;
                slots = (ncols + rounds - 1) / rounds;
            }
            double *Xc = (double *)c->buf("er_xc").ensure(sizeof(double) * (size_t)ncols * ldn);
            double *sl = (double *)c->buf("er_slots").ensure(sizeof(double) * (size_t)slots * 3 * ldn);
            // unit-weight test + diagonal, then the SELL-16 copy of L_reg
            auto *sdiag = (double *)c->buf("er_sell_diag").ensure(sizeof(double) * (n + 1));
            auto *uflag = (int32_t *)c->buf("er_unit_flag").ensure(sizeof(int32_t));
            const int64_t nbk = (n + kSell - 1) / kSell;
            auto *swid = (int32_t *)c->buf("er_sell_wid").ensure(sizeof(int32_t) * (nbk + 1));
            auto *soff = (int64_t *)c->buf("er_sell_off").ensure(sizeof(int64_t) * (nbk + 1));
            // unit-weight flags, diagonal, SELL slice widths / offsets: functions of L_reg,
            // i.e. of (graph, reg) -- computed and read back once (er_prepare's key)
            if (er.unit_key != er.prep_key) {
                int32_t one = 3;  // bit 0: unit weights, bit 1: diagonal = entries - 1 + 1e-6
                GS_HIP(hipMemcpyAsync(uflag, &one, sizeof(one), hipMemcpyHostToDevice, c->stream));
                if (n)
                    k_l_unit<<<grid_for(n, 256, 8192), 256, 0, c->stream>>>(lp, li, lv, n, sdiag, uflag);
                auto *scnt = (int64_t *)c->scratch[0].ensure(sizeof(int64_t) * (nbk + 1));
                GS_HIP(hipMemsetAsync(scnt, 0, sizeof(int64_t) * (nbk + 1), c->stream));
                if (nbk) k_sell_width<<<grid_for(nbk, 256, 4096), 256, 0, c->stream>>>(n, lp, swid, scnt);
                exclusive_scan_i64(c, scnt, soff, nbk + 1);
                er.sell_wid.assign((size_t)nbk, 0);
                GS_HIP(hipMemcpyAsync(&er.sell_sent, soff + nbk, sizeof(int64_t), hipMemcpyDeviceToHost,
                                      c->stream));
                GS_HIP(hipMemcpyAsync(&er.unit_flags, uflag, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
                if (nbk)
                    GS_HIP(hipMemcpyAsync(er.sell_wid.data(), swid, sizeof(int32_t) * nbk,
                                          hipMemcpyDeviceToHost, c->stream));
                GS_HIP(hipStreamSynchronize(c->stream));
                er.unit_key = er.prep_key;
            }
            const int64_t sent = er.sell_sent;
            int32_t unit = er.unit_flags;
            const int32_t dcount = (unit & 3) == 3 ? 1 : 0;
            unit &= 1;
            if (const char *e = getenv("GSPARSE_RES_UNIT")) unit = unit && atoi(e) != 0;
            long long *rprof = nullptr;
            if (getenv("GSPARSE_RES_PROF"))
                rprof = (long long *)c->buf("er_res_prof").ensure(8 * sizeof(long long));
            hipEvent_t t0 = nullptr;
            if (mode == 5) {
                int32_t dc = dcount;
                if (const char *e = getenv("GSPARSE_RES_DCOUNT")) dc = dc && atoi(e) != 0;
                if (n) GS_HIP(hipMemsetAsync(cp.iters + col0, 0, sizeof(int32_t) * ncols, c->stream));
                t0 = prof_begin(c);
                if (n)
                    cg_regres_solve(c, n, lp, li, lv, unit, dc, sdiag, Rr, er.ld, col0, ncols, maxiter,
                                    rtol, ch.count, ch.a, ch.len, Xc, ldn, cp.iters, slots, rprof);
                else
                    GS_HIP(hipMemsetAsync(cp.iters + col0, 0, sizeof(int32_t) * ncols, c->stream));
            } else {
            // longest row (the SELL block widths hold it) -> ELL width 4 / 8 / 12 / 16, else SELL
            int32_t maxw = 0;
            int sell_w = 8;
            {
                const std::vector<int32_t> &hw = er.sell_wid;
                for (int32_t v : hw) maxw = v > maxw ? v : maxw;
                // entries per row loaded at once: the smallest W in 6..8 that leaves at most
                // 1 in 10 of the 64-row tiles (a wave's rows, 4 slices) to the tail loop
                const int64_t ntl = (nbk + 3) / 4;
                for (int wc = 6; wc <= 8; ++wc) {
                    int64_t over = 0;
                    for (int64_t t = 0; t < ntl; ++t) {
                        int32_t m = 0;
                        for (int64_t b = 4 * t; b < 4 * t + 4 && b < nbk; ++b) m = hw[b] > m ? hw[b] : m;
                        over += m > wc;
                    }
                    sell_w = wc;
                    if (over * 10 <= ntl) break;
                }
            }
            // (measured on the Roman layout: SELL-16 40 us per column-iteration vs ELL-12 48 us --
            // the padded index loads cost more than the dependent block-offset load saves)
            int ew = maxw <= 4 ? 4 : maxw <= 8 ? 8 : maxw <= 12 ? 12 : maxw <= 16 ? 16 : 0;
            const char *ee = getenv("GSPARSE_RES_ELL");
            if (!ee || atoi(ee) == 0) ew = 0;
            const int64_t lde = (n + 63) & ~(int64_t)63;
            int32_t *ecol = nullptr;
            double *evalp = nullptr;
            if (ew && n) {
                ecol = (int32_t *)c->buf("er_ell_col").ensure(sizeof(int32_t) * (size_t)ew * lde);
                if (!unit) evalp = (double *)c->buf("er_ell_val").ensure(sizeof(double) * (size_t)ew * lde);
                k_ell_fill<<<grid_for(n, 256, 16384), 256, 0, c->stream>>>(n, ew, lde, lp, li, lv, ecol,
                                                                          evalp);
            }
            auto *scol = (int32_t *)c->buf("er_sell_col").ensure(sizeof(int32_t) * (sent + 1));
            double *sval = unit ? nullptr
                                : (double *)c->buf("er_sell_val").ensure(sizeof(double) * (sent + 1));
            GS_HIP(hipMemsetAsync(scol, 0xff, sizeof(int32_t) * (sent + 1), c->stream));
            if (nbk)
                k_sell_fill<<<grid_for(n, 256, 16384), 256, 0, c->stream>>>(
                    n, lp, li, lv, soff, swid, scol, sval);
            GS_HIP(hipGetLastError());
            ResArgs ra{n, er.ld, ldn, col0, ncols, lp, li, lv, Rr, Xc, sl, ca, cl, maxiter, rtol,
                       cp.iters, soff, swid, scol, sval, sdiag, ecol, evalp, lde, 0, 0, rprof,
                       dcount};
            if (const char *e = getenv("GSPARSE_RES_DCOUNT")) ra.dcount = ra.dcount && atoi(e) != 0;
            // q mirror in LDS: what the 160 KiB leave after the static 16 KiB
            // dynamic LDS (140 KiB next to the 16 KiB chain table): the SELL slice table
            // (8 B per 16 rows, when the offsets fit int32) and a mirror of q's first rows
            size_t lds = 140 * 1024;
            ra.nstab = (sent < (int64_t)1 << 31 && (size_t)nbk * 8 <= lds / 4) ? nbk : 0;
            if (const char *e = getenv("GSPARSE_RES_STAB")) if (atoi(e) == 0) ra.nstab = 0;
            lds -= (size_t)ra.nstab * 8;
            int64_t qlmax = (int64_t)(lds / 8);
            if (const char *e = getenv("GSPARSE_RES_QLDS")) qlmax = atoi(e) ? qlmax : 0;
            ra.ql = n < qlmax ? n : qlmax;
            const size_t dyn = sizeof(double) * (size_t)ra.ql + 8 * (size_t)ra.nstab + 8;
            t0 = prof_begin(c);
#define GS_RES(B, W, C, U, E)                                                                  \
    do {                                                                                        \
        GS_HIP(hipFuncSetAttribute((const void *)k_cg_resident<B, W, C, U, E>,                  \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));     \
        k_cg_resident<B, W, C, U, E><<<(unsigned)slots, kResThreads, dyn, c->stream>>>(ra, ch); \
    } while (0)
            // SpMV rows per thread-trip and entries loaded at once: 2 x W, W from the slice
            // widths above (Roman: W = 7, 419 ms per step vs 439 with 8 and 427 with 6;
            // 4 x 4 was slower, its rows wider than 4 take the tail loop)
            int rbw = 20 + sell_w;
            if (const char *e = getenv("GSPARSE_RES_RBW")) rbw = atoi(e) == 44 ? 44 : atoi(e) == 27 ? 27 : atoi(e) == 26 ? 26 : 28;
#define GS_RES_U(E)                                                  \
    do {                                                             \
        if (rbw == 28) {                                             \
            if (unit) GS_RES(2, 8, 16, true, E); else GS_RES(2, 8, 16, false, E); \
        } else if (rbw == 27) {                                      \
            if (unit) GS_RES(2, 7, 16, true, E); else GS_RES(2, 7, 16, false, E); \
        } else if (rbw == 26) {                                      \
            if (unit) GS_RES(2, 6, 16, true, E); else GS_RES(2, 6, 16, false, E); \
        } else {                                                     \
            if (unit) GS_RES(4, 4, 16, true, E); else GS_RES(4, 4, 16, false, E); \
        }                                                            \
    } while (0)
            if (n) {
                if (ew == 4) GS_RES_U(4);
                else if (ew == 8) GS_RES_U(8);
                else if (ew == 12) GS_RES_U(12);
                else if (ew == 16) GS_RES_U(16);
                else GS_RES_U(0);
            } else {
                GS_HIP(hipMemsetAsync(cp.iters + col0, 0, sizeof(int32_t) * ncols, c->stream));
            }
#undef GS_RES_U
#undef GS_RES
            }
            GS_HIP(hipGetLastError());
            prof_end(c, t0, mode == 5 ? "cg_reg" : "cg_res", 0.0);
            const bool prof_rec = c->profiling && !c->pending.empty();
            if (n)
                k_cols_to_rows<<<dim3((unsigned)((n + 31) / 32), (unsigned)((ncols + 31) / 32)), 256, 0,
                                 c->stream>>>(Xc, ldn, n, col0, ncols, X, er.ld);
            GS_HIP(hipGetLastError());
            GS_HIP(hipMemcpyAsync(er.iters.ptr, cp.iters, sizeof(int32_t) * k, hipMemcpyDeviceToDevice,
                                  c->stream));
            if (prof_rec) {
                // algorithmic bytes (SURVEY 8(d) B_ER): 8 (nnz(L_reg) + 10 n) per column and
                // iteration, + b in and x out per column; the iterations are summed on the
                // device and read when the profile is flushed
                ProfPending &pp = c->pending.back();
                pp.bytes = 16.0 * n * ncols;
                pp.its_slot = (int64_t)c->pending.size() - 1;
                pp.its_bytes = 8.0 * ((double)er.lnnz + 10.0 * n);
                auto *slots = c->buf("prof_its").ensure(sizeof(int64_t) * kProfPendingMax);
                k_sum_i32<<<1, 256, 0, c->stream>>>(cp.iters + col0, ncols, (int64_t *)slots + pp.its_slot);
            }
            sync_if_needed(c);
            if (rprof) {
                long long h[5];
                GS_HIP(hipMemcpy(h, rprof, sizeof(h), hipMemcpyDeviceToHost));
                fprintf(stderr,
                        "[gsparse] resident CG, workgroup 0 (us): p %.1f spmv %.1f pq %.1f upd %.1f finish %.1f\n",
                        h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0, h[4] / 100.0);
            }
            er.pcur = 0;
            er.solved = true;
            std::fill(er.col_solved.begin() + col0, er.col_solved.begin() + col1, 1);
            return;
        }
        GS_HIP(hipMemsetAsync(cp.nactive, 0, sizeof(int32_t), c->stream));
        // ||b|| and rho_0 (r = b.copy())
        if (cpl == 2) k_dot_acc<2, 4><<<grid, block, 0, c->stream>>>(G, ch, Rr, Rr, acc);
        else k_dot_acc<1, 4><<<grid, block, 0, c->stream>>>(G, ch, Rr, Rr, acc);
        k_fin_init<<<fgrid, 256, 0, c->stream>>>(G, ca, cl, ch.count, acc, Rr, rtol, cp.bn,
                                                  cp.atol, cp.rho, cp.active, cp.iters, cp.xstep,
                                                  cp.nactive);
        if (n)
            k_x_init<<<grid_for(n * ncols, 256, 65536), 256, 0, c->stream>>>(G, Rr, cp.bn, X);
        GS_HIP(hipGetLastError());
        int cur = 0;
        int32_t it_last = -1;
        for (int32_t it = 0; it < maxiter; ++it) {
            if (it % 8 == 0) {
                int32_t na = 0;
                GS_HIP(hipMemcpyAsync(&na, cp.nactive, sizeof(int32_t), hipMemcpyDeviceToHost,
                                      c->stream));
                GS_HIP(hipStreamSynchronize(c->stream));
                if (na == 0) break;
            }
            double *Pold = P[cur], *Pnew = P[cur ^ 1];
            hipEvent_t t0 = prof_begin(c);
#define GS_PQU(F, C, S, U)                                                                     \
    k_cg_pq<F, C, S, U><<<grid, block, 0, c->stream>>>(G, ch, lp, li, lv, Rr, Pold, Pnew, X,     \
                                                      qside, Qfull, cp.rho, cp.rho_prev,        \
                                                      cp.alpha, cp.active, cp.xstep, it, acc)
#define GS_PQ(F, C, S)                 \
    do {                               \
        if (ru == 1) GS_PQU(F, C, S, 1); \
        else if (ru == 2) GS_PQU(F, C, S, 2); \
        else if (ru == 4) GS_PQU(F, C, S, 4); \
        else GS_PQU(F, C, S, 8);       \
    } while (0)
#define GS_PQ_S(F, C) \
    if (storeq) GS_PQ(F, C, true); else GS_PQ(F, C, false)
#define GS_Q(C) k_cg_q<C><<<grid, block, 0, c->stream>>>(G, ch, lp, li, lv, Pnew, Qfull, cp.active, acc)
            if (mode >= 2) {
                const dim3 pg((unsigned)(((ncols + 1) / 2 + 255) / 256),
                              (unsigned)((n + kFlatRows - 1) / kFlatRows));
                if (it == 0)
                    k_cg_p_flat<true><<<pg, 256, 0, c->stream>>>(G, Rr, Pold, Pnew, X, cp.rho,
                                                                 cp.rho_prev, cp.alpha, cp.active,
                                                                 cp.xstep, it);
                else
                    k_cg_p_flat<false><<<pg, 256, 0, c->stream>>>(G, Rr, Pold, Pnew, X, cp.rho,
                                                                  cp.rho_prev, cp.alpha, cp.active,
                                                                  cp.xstep, it);
            }
            if (mode >= 2) {
                prof_end(c, t0, "cg_p", (it == 0 ? 16.0 : 40.0) * n * ncols);
                t0 = prof_begin(c);
                if (mode == 2) {
                    if (cpl == 2) GS_Q(2); else GS_Q(1);
                    prof_end(c, t0, "cg_q", (24.0 * n + 8.0 * lnz) * ncols);
                } else {
                    // 4 rows per wave, 128 columns: best of {1..64} x {64, 128} on ogbn-arxiv size
                    const int64_t rpw = 4;
                    const int scpl = 2;
                    CgGeom GS = G;
                    GS.ncb = (int32_t)((ncols + 64 * scpl - 1) / (64 * scpl));
                    const int64_t ntiles = (n + rpw - 1) / rpw;
                    const unsigned sg = (unsigned)((GS.ncb * ntiles + 3) / 4);
                    if (scpl == 2)
                        k_spmv<2><<<sg, 256, 0, c->stream>>>(GS, rpw, ntiles, lp, li, lv, Pnew, Qfull, cp.active);
                    else
                        k_spmv<1><<<sg, 256, 0, c->stream>>>(GS, rpw, ntiles, lp, li, lv, Pnew, Qfull, cp.active);
                    prof_end(c, t0, "cg_spmv", (8.0 * n + 8.0 * lnz) * ncols);
                    t0 = prof_begin(c);
                    if (cpl == 2) k_dot_acc<2, 4><<<grid, block, 0, c->stream>>>(G, ch, Pnew, Qfull, acc);
                    else k_dot_acc<1, 4><<<grid, block, 0, c->stream>>>(G, ch, Pnew, Qfull, acc);
                    prof_end(c, t0, "cg_dot", 16.0 * n * ncols);
                }
            } else if (it == 0) {
                if (cpl == 2) { GS_PQ_S(true, 2); } else { GS_PQ_S(true, 1); }
            } else {
                if (cpl == 2) { GS_PQ_S(false, 2); } else { GS_PQ_S(false, 1); }
            }
#undef GS_Q
#undef GS_PQ_S
#undef GS_PQ
#undef GS_PQU
            if (mode < 2) prof_end(c, t0, "cg_pq", it == 0 ? bytes_pq0 : bytes_pq);
            k_fin_pq<<<fgrid, 256, 0, c->stream>>>(G, ca, cl, ch.count, acc, Pnew, Qfull, qside, cp.rho,
                                                   cp.active, it,
                                                  cp.alpha, cp.xstep);
            t0 = prof_begin(c);
#define GS_UPDU(C, S, U)                                                                    \
    k_cg_upd<C, S, U><<<grid, block, 0, c->stream>>>(G, ch, lp, li, lv, Pnew, Qfull, Rr,      \
                                                     cp.alpha, cp.active, acc)
#define GS_UPD(C, S)                  \
    do {                              \
        if (ru == 1) GS_UPDU(C, S, 1); \
        else if (ru == 2) GS_UPDU(C, S, 2); \
        else if (ru == 4) GS_UPDU(C, S, 4); \
        else GS_UPDU(C, S, 8);        \
    } while (0)
            if (cpl == 2) {
                if (storeq) GS_UPD(2, true); else GS_UPD(2, false);
            } else {
                if (storeq) GS_UPD(1, true); else GS_UPD(1, false);
            }
#undef GS_UPD
#undef GS_UPDU
            prof_end(c, t0, "cg_upd", bytes_upd);
            k_fin_rr<<<fgrid, 256, 0, c->stream>>>(G, ca, cl, ch.count, acc, Rr, it, cp.rho,
                                                   cp.rho_prev, cp.atol,
                                                  cp.active, cp.iters, cp.nactive);
            GS_HIP(hipGetLastError());
            cur ^= 1;
            it_last = it;
        }
        // the x update of the last executed iteration (P[cur] holds its p)
        if (it_last >= 0 && n)
            k_x_flush<<<grid_for(n * ncols, 256, 65536), 256, 0, c->stream>>>(G, P[cur], cp.alpha,
                                                                              cp.xstep, it_last, X);
        GS_HIP(hipGetLastError());
        er.pcur = cur;
        GS_HIP(hipMemcpyAsync(er.iters.ptr, cp.iters, sizeof(int32_t) * k, hipMemcpyDeviceToDevice,
                              c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
        er.solved = true;
        std::fill(er.col_solved.begin() + col0, er.col_solved.begin() + col1, 1);
    });
}

int gs_er_scores(gs_ctx *c, int64_t col0, int64_t col1, int64_t e0, int64_t e1, int finalize,
                 double *out, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.solved, GS_ESTATE, "gs_er_solve first");
        GS_CHECK(0 <= col0 && col0 <= col1 && col1 <= er.k, GS_EINVAL, "bad column range");
        GS_CHECK(0 <= e0 && e0 <= e1 && e1 <= c->g.nnz, GS_EINVAL, "bad edge range");
        GS_CHECK(er_cols_solved(er, col0, col1), GS_ESTATE,
                 "columns [%lld, %lld) were not all solved since gs_er_prepare", (long long)col0,
                 (long long)col1);
        GS_HIP(hipSetDevice(c->device));
        int64_t cnt = e1 - e0;
        double *dout = (double *)out_device(c, c->outbuf, out, sizeof(double) * cnt, loc);
        if (cnt) {
            hipEvent_t t0 = prof_begin(c);
            k_er_scores<<<grid_for(cnt, 64), 64, 0, c->stream>>>(
                c->g.rows.as<int32_t>(), c->g.indices.as<int32_t>(), er.X.as<double>(), er.ld, col0,
                col1, e0, e1, finalize, dout);
            GS_HIP(hipGetLastError());
            prof_end(c, t0, "er_scores", (16.0 * (col1 - col0) + 16.0) * cnt);
        }
        finish_out(c, out, dout, sizeof(double) * cnt, loc);
    });
}

int gs_er_copy_z(gs_ctx *c, int64_t col0, int64_t col1, double *out, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.solved, GS_ESTATE, "gs_er_solve first");
        GS_CHECK(out, GS_EINVAL, "out is NULL");
        GS_CHECK(0 <= col0 && col0 <= col1 && col1 <= er.k, GS_EINVAL, "bad column range");
        GS_CHECK(er_cols_solved(er, col0, col1), GS_ESTATE,
                 "columns [%lld, %lld) were not all solved since gs_er_prepare", (long long)col0,
                 (long long)col1);
        GS_HIP(hipSetDevice(c->device));
        const int64_t nc = col1 - col0;
        if (nc && er.n)
            GS_HIP(hipMemcpy2DAsync(out, sizeof(double) * nc, er.X.as<double>() + col0,
                                    sizeof(double) * er.ld, sizeof(double) * nc, er.n,
                                    loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                                    c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

int gs_er_iterations(gs_ctx *c, int32_t *iters, int loc) {
    return guard([&] {
        GS_CHECK(c, GS_EINVAL, "null context");
        ErState &er = c->er;
        GS_CHECK(er.solved, GS_ESTATE, "gs_er_solve first");
        GS_HIP(hipMemcpyAsync(iters, er.iters.ptr, sizeof(int32_t) * er.k,
                              loc == GS_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                              c->stream));
        GS_HIP(hipStreamSynchronize(c->stream));
    });
}

int gs_er_split(int64_t k, int32_t parts, int64_t *bounds) {
    return guard([&] {
        GS_CHECK(parts >= 1 && (parts & (parts - 1)) == 0, GS_EINVAL, "parts must be a power of 2");
        GS_CHECK(bounds, GS_EINVAL, "bounds is NULL");
        std::vector<int64_t> b = {0, k};
        for (int32_t p = 1; p < parts; p *= 2) {
            std::vector<int64_t> nb = {0};
            for (size_t i = 0; i + 1 < b.size(); ++i) {
                int64_t lo = b[i], len = b[i + 1] - b[i];
                GS_CHECK(len > 128, GS_EINVAL,
                         "k=%lld too small to split %d ways along the pairwise tree",
                         (long long)k, parts);
                int64_t n2 = len / 2;
                n2 -= n2 % 8;
                nb.push_back(lo + n2);
                nb.push_back(b[i + 1]);
            }
            b.swap(nb);
        }
        for (size_t i = 0; i < b.size(); ++i) bounds[i] = b[i];
    });
}

}  // extern "C"
