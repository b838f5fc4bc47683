/*
 * oracle.c -- CPU restatement of the reference edge-scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline -- never as the product path.
 *
 * Every function restates one reference step, cited as
 * /root/reference/src/sparsification/<file>:<line>.  The reference is pure
 * Python over NumPy/SciPy/NetworkX; the arithmetic contracts restated here
 * were pinned against golden vectors produced by the reference itself
 * (tests/golden/make_golden.py, tests/test_oracle_golden.py).
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off: no FMA contraction,
 * every product is rounded before it is summed, as in SciPy/NumPy's C loops).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------------- */
/* Jaccard: metrics.py:43-62.
 *   Ab = (A>0); deg = rowsum(Ab); inter = (Ab@Ab)[u,v] = |out(u) ∩ in(v)|;
 *   union = deg[u]+deg[v]-inter; score = inter/union if union>0 else 0.
 * CSR is canonical (sorted, duplicate-free); (tp, ti) is its transpose
 * (in-neighbour lists, sorted). Counts are exact integers, then ONE fp64
 * division -- bit-identical to the reference's float64 counts. */
void oracle_jaccard(int64_t n, const int64_t *ip, const int32_t *ix,
                    const int64_t *tp, const int32_t *ti, double *out) {
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int32_t v = ix[e];
            int64_t a = ip[u], ae = ip[u + 1], b = tp[v], be = tp[v + 1];
            int64_t inter = 0;
            while (a < ae && b < be) {
                int32_t x = ix[a], y = ti[b];
                if (x == y) { ++inter; ++a; ++b; }
                else if (x < y) ++a;
                else ++b;
            }
            double du = (double)(ip[u + 1] - ip[u]);
            double dv = (double)(ip[v + 1] - ip[v]);
            double uni = du + dv - (double)inter;
            out[e] = uni > 0 ? (double)inter / uni : 0.0;
        }
    }
}

/* The same per-edge merge for the entries of rows [r0, r1) only (out indexed by
 * CSR position): bench.py's bounded CPU-baseline sample on R-MAT graphs. */
void oracle_jaccard_rows(const int64_t *ip, const int32_t *ix, const int64_t *tp,
                         const int32_t *ti, int64_t r0, int64_t r1, double *out) {
    for (int64_t u = r0; u < r1; ++u) {
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int32_t v = ix[e];
            int64_t a = ip[u], ae = ip[u + 1], b = tp[v], be = tp[v + 1];
            int64_t inter = 0;
            while (a < ae && b < be) {
                int32_t x = ix[a], y = ti[b];
                if (x == y) { ++inter; ++a; ++b; }
                else if (x < y) ++a;
                else ++b;
            }
            double du = (double)(ip[u + 1] - ip[u]);
            double dv = (double)(ip[v + 1] - ip[v]);
            double uni = du + dv - (double)inter;
            out[e] = uni > 0 ? (double)inter / uni : 0.0;
        }
    }
}

/* Adamic-Adar: metrics.py:99-119.
 *   c_w = 1/sqrt(max(log(deg_w+1),1e-10)) (computed by NumPy, passed in);
 *   AA[u,v] = sum over w in out(u) ∩ out(v) of c_w*c_w, accumulated from 0.0
 *   in DESCENDING w: W = Ab@diag(c) comes out of SciPy csr_matmat with each
 *   row's columns in linked-list (= descending) order, and W@W.T folds row u
 *   of W in that stored order. */
void oracle_adamic_adar(int64_t n, const int64_t *ip, const int32_t *ix,
                        const double *c, double *out) {
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int32_t v = ix[e];
            int64_t a = ip[u + 1] - 1, b = ip[v + 1] - 1;
            double s = 0.0;
            while (a >= ip[u] && b >= ip[v]) {
                int32_t x = ix[a], y = ix[b];
                if (x == y) { double p = c[x] * c[x]; s = s + p; --a; --b; }
                else if (x > y) --a;
                else --b;
            }
            out[e] = s;
        }
    }
}

/* NumPy pairwise summation (numpy/_core/src/umath/loops_utils.h.src,
 * pairwise_sum_@TYPE@): n<8 sequential from 0; n<=128 eight strided
 * accumulators combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail;
 * else split at n/2 rounded down to a multiple of 8. */
static float pw_sum_f32(const float *a, int64_t n) {
    if (n < 8) {
        float r = 0.f;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        float r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pw_sum_f32(a, n2) + pw_sum_f32(a + n2, n - n2);
    }
}

static double pw_sum_f64(const double *a, int64_t n) {
    if (n < 8) {
        double r = 0.;
        for (int64_t i = 0; i < n; ++i) r += a[i];
        return r;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pw_sum_f64(a, n2) + pw_sum_f64(a + n2, n - n2);
    }
}

double oracle_pairwise_sum_f64(const double *a, int64_t n) { return pw_sum_f64(a, n); }
float oracle_pairwise_sum_f32(const float *a, int64_t n) { return pw_sum_f32(a, n); }

/* Feature cosine, float32 features: metrics.py:344-358.
 *   norm_i = sqrt(0 + pw_sum(x_i*x_i)); xn = x / max(norm, f32(1e-10));
 *   s_e = pw_sum(xn_u*xn_v); max(s, 0); -> float64. */
void oracle_feature_cosine_f32(int64_t n, int64_t f, const int64_t *ip, const int32_t *ix,
                               const float *x, double *out) {
    float *xn = (float *)malloc(sizeof(float) * (size_t)(n * f));
    float *tmp = (float *)malloc(sizeof(float) * (size_t)(f > 0 ? f : 1));
    const float floor_ = (float)1e-10;
    for (int64_t i = 0; i < n; ++i) {
        const float *r = x + i * f;
        for (int64_t k = 0; k < f; ++k) tmp[k] = r[k] * r[k];
        float nrm = sqrtf(0.f + pw_sum_f32(tmp, f));
        if (!(nrm >= floor_)) nrm = (nrm != nrm) ? nrm : floor_;  /* np.maximum propagates NaN */
        for (int64_t k = 0; k < f; ++k) xn[i * f + k] = r[k] / nrm;
    }
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int64_t v = ix[e];
            for (int64_t k = 0; k < f; ++k) tmp[k] = xn[u * f + k] * xn[v * f + k];
            float s = 0.f + pw_sum_f32(tmp, f);
            if (!(s >= 0.f)) s = (s != s) ? s : 0.f;
            out[e] = (double)s;
        }
    }
    free(xn);
    free(tmp);
}

void oracle_feature_cosine_f64(int64_t n, int64_t f, const int64_t *ip, const int32_t *ix,
                               const double *x, double *out) {
    double *xn = (double *)malloc(sizeof(double) * (size_t)(n * f));
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(f > 0 ? f : 1));
    for (int64_t i = 0; i < n; ++i) {
        const double *r = x + i * f;
        for (int64_t k = 0; k < f; ++k) tmp[k] = r[k] * r[k];
        double nrm = sqrt(0. + pw_sum_f64(tmp, f));
        if (!(nrm >= 1e-10)) nrm = (nrm != nrm) ? nrm : 1e-10;
        for (int64_t k = 0; k < f; ++k) xn[i * f + k] = r[k] / nrm;
    }
    for (int64_t u = 0; u < n; ++u) {
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int64_t v = ix[e];
            for (int64_t k = 0; k < f; ++k) tmp[k] = xn[u * f + k] * xn[v * f + k];
            double s = 0. + pw_sum_f64(tmp, f);
            if (!(s >= 0.)) s = (s != s) ? s : 0.;
            out[e] = s;
        }
    }
    free(xn);
    free(tmp);
}

/* ---------------------------------------------------------------------- */
/* ApproxER CG.  Everything follows SciPy 1.15 cg
 * (scipy/sparse/linalg/_isolve/iterative.py) as called at metrics.py:284-289:
 * x0=0, r=b, stop at loop top if ||r|| < rtol*||b||, z=r, rho=r.r,
 * p = beta*p + z (two roundings), q = L_reg p (csr_matvec: per-row fold from
 * 0.0, ascending column, no FMA), alpha = rho/(p.q), x += fl(alpha*p),
 * r -= fl(alpha*q); ||v|| = sqrt(v.v) (numpy.linalg.norm -> dot).
 *
 * Every dot product is np.dot -> OpenBLAS ddot.  Its reduction order was
 * pinned empirically against np.dot on this image's OpenBLAS 0.3.29
 * (SkylakeX kernel), bit-exact for every n tried (1..300, 1e3..1e5):
 *   - threads: for n <= 10000 one chunk; else the vector is split over T
 *     threads, chunk width = ceil(remaining / threads_left), and the chunk
 *     results are summed left to right from 0.0;
 *   - per chunk of length L: n1 = L & -16, n32 = n1 & ~31; 32 FMA
 *     accumulators a[j] over elements j, j+32, ... < n32; fold
 *     b[4q+l] = a[8q+l] + a[8q+4+l]; if n1 > n32 one more 16-block
 *     b[4q+l] = fma(x, y, b[4q+l]); c[l] = ((b[l]+b[4+l])+b[8+l])+b[12+l];
 *     dot = (c0+c2) + (c1+c3) (0.0 when n1 == 0); then the tail
 *     dot = fma(x[i], y[i], dot) for i >= n1.
 * Y (n x k, row-major) in, Z (n x k, row-major) out; b == 0 -> Z col = 0.
 * iters_out[c] receives the number of iterations column c ran. */
static double ddot_chunk(const double *x, const double *y, int64_t L) {
    int64_t n1 = L & -16, n32 = n1 & ~(int64_t)31, i = 0;
    double dot = 0.0;
    if (n1) {
        double a[32], b[16], c[4];
        for (int j = 0; j < 32; ++j) a[j] = 0.0;
        for (; i < n32; i += 32)
            for (int j = 0; j < 32; ++j) a[j] = fma(x[i + j], y[i + j], a[j]);
        for (int q = 0; q < 4; ++q)
            for (int l = 0; l < 4; ++l) b[4 * q + l] = a[8 * q + l] + a[8 * q + 4 + l];
        for (; i < n1; i += 16)
            for (int j = 0; j < 16; ++j) b[j] = fma(x[i + j], y[i + j], b[j]);
        for (int l = 0; l < 4; ++l) c[l] = ((b[l] + b[4 + l]) + b[8 + l]) + b[12 + l];
        dot = (c[0] + c[2]) + (c[1] + c[3]);
    }
    for (i = n1; i < L; ++i) dot = fma(y[i], x[i], dot);
    return dot;
}

double oracle_ddot(const double *x, const double *y, int64_t n, int32_t threads) {
    if (n <= 10000 || threads <= 1) return ddot_chunk(x, y, n);
    double s = 0.0;
    int64_t lo = 0, rem = n;
    for (int32_t t = threads; t > 0 && rem > 0; --t) {
        int64_t w = (rem + t - 1) / t;
        s = s + ddot_chunk(x + lo, y + lo, w);
        lo += w;
        rem -= w;
    }
    return s;
}

void oracle_cg(int64_t n, const int64_t *lp, const int32_t *li, const double *lv,
               int64_t k, const double *Y, int32_t maxiter, double rtol, int32_t threads,
               double *Z, int32_t *iters_out) {
    double *b = (double *)malloc(sizeof(double) * (size_t)n);
    double *x = (double *)malloc(sizeof(double) * (size_t)n);
    double *r = (double *)malloc(sizeof(double) * (size_t)n);
    double *p = (double *)malloc(sizeof(double) * (size_t)n);
    double *q = (double *)malloc(sizeof(double) * (size_t)n);
    for (int64_t c = 0; c < k; ++c) {
        for (int64_t i = 0; i < n; ++i) { b[i] = Y[i * k + c]; x[i] = 0.0; r[i] = b[i]; }
        double bn = sqrt(oracle_ddot(b, b, n, threads));
        int32_t it = 0;
        if (bn != 0.0) {
            double atol = rtol * bn;
            double rho_prev = 0.0;
            for (it = 0; it < maxiter; ++it) {
                double rho = oracle_ddot(r, r, n, threads);
                if (sqrt(rho) < atol) break;
                if (it > 0) {
                    double beta = rho / rho_prev;
                    for (int64_t i = 0; i < n; ++i) { double t = p[i] * beta; p[i] = t + r[i]; }
                } else {
                    memcpy(p, r, sizeof(double) * (size_t)n);
                }
                for (int64_t i = 0; i < n; ++i) {
                    double s = 0.0;
                    for (int64_t e = lp[i]; e < lp[i + 1]; ++e) { double t = lv[e] * p[li[e]]; s = s + t; }
                    q[i] = s;
                }
                double alpha = rho / oracle_ddot(p, q, n, threads);
                for (int64_t i = 0; i < n; ++i) {
                    double t = alpha * p[i]; x[i] = x[i] + t;
                    double u = alpha * q[i]; r[i] = r[i] - u;
                }
                rho_prev = rho;
            }
        }
        for (int64_t i = 0; i < n; ++i) {
            double v = x[i];
            if (v != v || isinf(v)) v = 0.0;  /* nan_to_num(nan=0,posinf=0,neginf=0) */
            Z[i * k + c] = v;
        }
        if (iters_out) iters_out[c] = it;
    }
    free(b); free(x); free(r); free(p); free(q);
}

/* r_eff = sum_c (Z[u,c]-Z[v,c])^2 (NumPy pairwise over k, fp64), then
 * nan_to_num(1e-10) and max(.,1e-10): metrics.py:292-297. */
void oracle_er_from_z(int64_t n, const int64_t *ip, const int32_t *ix, int64_t k,
                      const double *Z, double *out) {
    double *tmp = (double *)malloc(sizeof(double) * (size_t)(k > 0 ? k : 1));
    for (int64_t u = 0; u < n; ++u)
        for (int64_t e = ip[u]; e < ip[u + 1]; ++e) {
            int64_t v = ix[e];
            for (int64_t c = 0; c < k; ++c) { double d = Z[u * k + c] - Z[v * k + c]; tmp[c] = d * d; }
            double s = 0.0 + pw_sum_f64(tmp, k);
            if (s != s || isinf(s)) s = 1e-10;
            out[e] = s > 1e-10 ? s : 1e-10;
        }
    free(tmp);
}

/* ---------------------------------------------------------------------- */
/* Metric backbone: metric_backbone.py:59-111.
 * G = undirected graph of the edge_index columns with u<v, weight = min over
 * duplicates (:70-79).  For every column idx=(u,v): d = Dijkstra distance
 * u->v in G (sums left-folded from u, as networkx _dijkstra_multisource
 * does), keep iff d == inf or w[idx] <= d + eps (:97-111).
 * Restated as one bounded Dijkstra per distinct row u: it stops once every
 * target of u is settled or the frontier passes the largest target weight
 * (an unsettled target then has d > w >= w - eps, i.e. it is kept). */
typedef struct { double d; int32_t v; } hent;

static void heap_push(hent *h, int64_t *hn, double d, int32_t v) {
    int64_t i = (*hn)++;
    while (i > 0) {
        int64_t p = (i - 1) >> 1;
        if (h[p].d <= d) break;
        h[i] = h[p];
        i = p;
    }
    h[i].d = d; h[i].v = v;
}

static hent heap_pop(hent *h, int64_t *hn) {
    hent top = h[0];
    hent last = h[--(*hn)];
    int64_t i = 0, n = *hn;
    for (;;) {
        int64_t l = 2 * i + 1;
        if (l >= n) break;
        int64_t m = (l + 1 < n && h[l + 1].d < h[l].d) ? l + 1 : l;
        if (h[m].d >= last.d) break;
        h[i] = h[m];
        i = m;
    }
    if (n > 0) h[i] = last;
    return top;
}

/* gp/gi/gw: symmetric CSR of G (built by the caller from the u<v columns,
 * min weight over duplicates).  rows/cols/w: the E edge_index columns.
 * order/optr: columns grouped by row (order = column ids sorted by row). */
/* sel/nsel: the source rows to decide (sel == NULL: every row 0..n-1); the
 * columns of other rows are left untouched in keep */
static int64_t backbone_rows(int64_t n, const int64_t *gp, const int32_t *gi, const double *gw,
                             const int64_t *cols, const double *w, double eps,
                             const int64_t *order, const int64_t *optr, const int64_t *sel,
                             int64_t nsel, uint8_t *keep, int64_t *relax_out) {
    double *dist = (double *)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
    uint8_t *done = (uint8_t *)calloc((size_t)(n > 0 ? n : 1), 1);
    uint8_t *tgt = (uint8_t *)calloc((size_t)(n > 0 ? n : 1), 1);
    int64_t cap = gp[n] + 16;
    hent *h = (hent *)malloc(sizeof(hent) * (size_t)cap);
    int32_t *touched = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
    int64_t relax = 0;
    for (int64_t i = 0; i < n; ++i) dist[i] = INFINITY;
    for (int64_t si = 0; si < (sel ? nsel : n); ++si) {
        const int64_t u = sel ? sel[si] : si;
        if (u < 0 || u >= n || optr[u] == optr[u + 1]) continue;
        double wmax = -INFINITY;
        int64_t ntg = 0;
        for (int64_t j = optr[u]; j < optr[u + 1]; ++j) {
            int64_t idx = order[j];
            int64_t v = cols[idx];
            if (!tgt[v]) { tgt[v] = 1; ++ntg; }
            if (w[idx] > wmax) wmax = w[idx];
        }
        int64_t nt = 0, hn = 0;
        dist[u] = 0.0; touched[nt++] = (int32_t)u;
        heap_push(h, &hn, 0.0, (int32_t)u);
        while (hn > 0 && ntg > 0) {
            hent t = heap_pop(h, &hn);
            if (done[t.v]) continue;
            if (t.d > wmax) break;
            done[t.v] = 1;
            if (tgt[t.v]) --ntg;
            for (int64_t e = gp[t.v]; e < gp[t.v + 1]; ++e) {
                int32_t y = gi[e];
                ++relax;
                if (done[y]) continue;
                double nd = t.d + gw[e];
                if (nd < dist[y]) {
                    if (dist[y] == INFINITY) touched[nt++] = y;
                    dist[y] = nd;
                    if (hn >= cap) { cap *= 2; h = (hent *)realloc(h, sizeof(hent) * (size_t)cap); }
                    heap_push(h, &hn, nd, y);
                }
            }
        }
        for (int64_t j = optr[u]; j < optr[u + 1]; ++j) {
            int64_t idx = order[j];
            int64_t v = cols[idx];
            double d = done[v] ? dist[v] : INFINITY;  /* unsettled: d > w, kept either way */
            if (v == u) d = 0.0;
            keep[idx] = (d == INFINITY) || (w[idx] <= d + eps);
            tgt[v] = 0;
        }
        for (int64_t i = 0; i < nt; ++i) { dist[touched[i]] = INFINITY; done[touched[i]] = 0; }
    }
    if (relax_out) *relax_out = relax;
    free(dist); free(done); free(tgt); free(h); free(touched);
    return 0;
}

int64_t oracle_metric_backbone(int64_t n, const int64_t *gp, const int32_t *gi, const double *gw,
                               int64_t E, const int64_t *rows, const int64_t *cols,
                               const double *w, double eps, const int64_t *order,
                               const int64_t *optr, uint8_t *keep, int64_t *relax_out) {
    (void)E; (void)rows;
    return backbone_rows(n, gp, gi, gw, cols, w, eps, order, optr, NULL, 0, keep, relax_out);
}

/* The same decisions for the columns of the listed source rows only (the
 * sampled-row pin of large graphs: one bounded Dijkstra per listed row). */
int64_t oracle_metric_backbone_rows(int64_t n, const int64_t *gp, const int32_t *gi,
                                    const double *gw, const int64_t *cols, const double *w,
                                    double eps, const int64_t *order, const int64_t *optr,
                                    int64_t nsel, const int64_t *sel, uint8_t *keep,
                                    int64_t *relax_out) {
    return backbone_rows(n, gp, gi, gw, cols, w, eps, order, optr, sel, nsel, keep, relax_out);
}
