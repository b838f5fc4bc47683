// gs_cg_reg.hip -- host side of the register-resident CG (ApproxER mode 5): the
// ELL-8 copy of L_reg with p codes, the LDS plan, geometry and launch.  The kernel
// and its design notes are in gs_cg_reg.hpp.
#include "gs_cg_reg.hpp"

#ifndef GS_CG_XG
#define GS_CG_XG 0
#endif

namespace gs {

// ELL-8 copy of L_reg: overflow entry counts (rows longer than 8)
__global__ void k_ell8_count(int32_t n, const int64_t *__restrict__ lp, int64_t *__restrict__ cnt,
                             uint16_t *__restrict__ rlen) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t len = lp[i + 1] - lp[i];
        cnt[i] = len > 8 ? len - 8 : 0;
        rlen[i] = (uint16_t)len;
    }
}

// p code of column c: its LDS slot when c is in its chunk's LDS-resident prefix,
// else 0x8000 | c (chunk table: starts, lengths, prefixes, LDS bases).  A split part's
// table holds only its own chunks: columns outside them are global (other parts' rows)
__device__ __forceinline__ uint32_t p_code(int32_t c, int T, const int64_t *__restrict__ tab) {
    if (c < tab[0] || c >= tab[T - 1] + tab[kRegMaxChunks + T - 1]) return 0x8000u | (uint32_t)c;
    int t = 0;
    while (t + 1 < T && c >= tab[t + 1]) ++t;
    const int64_t o = c - tab[t];
    return o < tab[2 * kRegMaxChunks + t] ? (uint32_t)(tab[3 * kRegMaxChunks + t] + o)
                                          : 0x8000u | (uint32_t)c;
}

// diagonal slot index of row c: 2 tid + parity in k_cg_regres (dmul 2), tid in
// k_cg_regwide (dmul 1), G threads per chain:
// chain row s of chain (t, j) is slot s / G of thread g = s % G; a chunk's tail rows
// belong to g = 0 with parity 0
__device__ __forceinline__ int row_dslot(int32_t c, int T, const int64_t *__restrict__ tab, int G,
                                         int dmul, int32_t d0 = 0) {
    int t = 0;
    while (t + 1 < T && c >= tab[t + 1]) ++t;
    const int o = (int)(c - tab[t]), n32 = (int)(tab[kRegMaxChunks + t] & ~(int64_t)31);
    const bool in = o < n32;
    const int j = in ? (o & 31) : o - n32, g = in ? (o >> 5) % G : 0;
    const int par = in ? ((o >> 5) / G) & 1 : 0;
    const int chain = t * 32 + j, CW = 64 / G;
    const int tid = (chain / CW) * 64 + (chain % CW) + CW * g;
    if (dmul == 3) {  // k_cg_regwide's V2 two-per-chain layout (DBANK): bank of own p + 1
        const int lb = (int)tab[3 * kRegMaxChunks + t];
        const int s0 = d0 + (tid & ~31);
        return (tid & ~31) + ((lb + (tid & 31) + 1 - s0) & 31);
    }
    return dmul == 2 ? 2 * tid + par : tid;
}

// dslot0 >= 0 (unit form): the diagonal entry's code is the owner thread's diagonal
// slot dslot0 + tid instead of the row's p code
__global__ void k_ell8_fill(int32_t r0, int32_t n, int T, const int64_t *__restrict__ tab, uint32_t pad,
                            int G, int dmul, int32_t dslot0, const int64_t *__restrict__ lp,
                            const int32_t *__restrict__ li, const double *__restrict__ lv,
                            const int64_t *__restrict__ optr, uint4 *__restrict__ ell,
                            double *__restrict__ ellv, uint16_t *__restrict__ ocol,
                            double *__restrict__ oval, uint8_t *__restrict__ rflag) {
    for (int64_t i = r0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e0 = lp[i], len = lp[i + 1] - e0;
        const uint32_t dcode = dslot0 >= 0 ? (uint32_t)(dslot0 + row_dslot((int32_t)i, T, tab, G, dmul, dslot0)) : 0u;
        auto code = [&](int64_t e) -> uint32_t {
            return (dslot0 >= 0 && li[e] == i) ? dcode : p_code(li[e], T, tab);
        };
        uint32_t w[4] = {0, 0, 0, 0};
        bool glob = false;
        for (int k = 0; k < 8; ++k) {
            const uint32_t cc = k < len ? code(e0 + k) : pad;
            glob = glob || (cc & 0x8000u) != 0;
            w[k >> 1] |= cc << (16 * (k & 1));
            if (ellv) ellv[i * 8 + k] = k < len ? lv[e0 + k] : 0.0;
        }
        ell[i] = make_uint4(w[0], w[1], w[2], w[3]);
        if (rflag) rflag[i] = (uint8_t)((glob ? 1 : 0) | (len > 8 ? 2 : 0));
        for (int64_t k = 8; k < len; ++k) {
            ocol[optr[i] + k - 8] = (uint16_t)code(e0 + k);
            if (oval) oval[optr[i] + k - 8] = lv[e0 + k];
        }
    }
}

// threads per chain for T chunks on an NT-thread workgroup (power of two, 32 T G <= NT,
// G <= 8) and register row slots per thread (the chain rows); -1 when it does not apply
static int reg_geometry(int NT, int T, const int64_t *len, int &G) {
    if (T < 1 || 32 * T > NT) return -1;
    G = 1;
    while (G < 8 && 32 * T * (2 * G) <= NT) G *= 2;
    int64_t smax = 0;
    for (int t = 0; t < T; ++t) smax = std::max<int64_t>(smax, (len[t] & ~(int64_t)31) >> 5);
    return (int)((smax + G - 1) / G);
}

// workgroup size and slots: 512 threads (two waves per SIMD, k_cg_regwide) where the
// slots fit 44, else 256 threads (one wave per SIMD, 512 registers per lane,
// k_cg_regres) with up to 88.  GSPARSE_REG_NT=256 forces the one-wave form.
static bool reg_pick(int64_t n, int T, const int64_t *len, int &NT, int &G, int &R) {
    if (n <= 0 || n >= 0x8000) return false;
    int g = 0;
    const char *e = getenv("GSPARSE_REG_NT");
    const bool narrow_only = e && atoi(e) == 256;
    int r = narrow_only ? -1 : reg_geometry(512, T, len, g);
    if (r >= 0 && r <= 44) {
        NT = 512, G = g;
        R = r <= 16 ? 16 : r <= 24 ? 24 : r <= 32 ? 32 : 44;
        return true;
    }
    r = reg_geometry(256, T, len, g);
    if (r < 0 || r > 88) return false;
    NT = 256, G = g;
    R = r <= 24 ? 24 : r <= 48 ? 48 : r <= 64 ? 64 : 88;
    return true;
}

bool cg_regres_applies(int64_t n, int T, const int64_t *len) {
    int NT, G, R;
    return reg_pick(n, T, len, NT, G, R);
}

bool cg_regres_wide(int64_t n, int T, const int64_t *len) {
    int NT = 0, G, R;
    return reg_pick(n, T, len, NT, G, R) && NT == 512;
}

void cg_regres_solve(gs_ctx *c, int64_t n, const int64_t *lp, const int32_t *li, const double *lv,
                     int unit, int dcount, const double *diag, const double *Rr, int64_t ld,
                     int64_t col0, int64_t ncols, int32_t maxiter, double rtol, int T,
                     const int64_t *ha, const int64_t *hlen, double *Xc, int64_t ldn,
                     int32_t *iters, int64_t slots, long long *prof) {
    hipStream_t s = c->stream;
    int NT = 0, G = 0, rsel = 0;
    GS_CHECK(reg_pick(n, T, hlen, NT, G, rsel), GS_EUNSUPPORTED,
             "register-resident CG: n=%lld, %d chunks out of range", (long long)n, T);
    // LDS: p (each chunk's LDS-resident prefix, in chunk order), the zero and scratch
    // slots, (one-wave form) 2 diagonal slots per thread, 6 x 32 T doubles of chain
    // sums / tail rows, the chunk table
    const int nch = 32 * T;
    const bool ufast = unit && dcount;  // the unit kernels derive every diagonal from the entry count
    // (512 threads, two per chain, unit: the diagonal slots bank-permuted -- the same
    // condition as k_cg_regwide's DBANK = GS_CG_V2 && UNIT && G == 2, so an A/B build with
    // -DGS_CG_V2=0 codes the diagonal where its kernel reads it)
    const bool dbank = GS_CG_V2 && NT == 512 && G == 2 && ufast;
    const int dsl = NT == 256 ? 2 * NT : ufast ? NT : 0;
    const size_t lds_max = 160 * 1024;
    const int64_t cap =
        (int64_t)((lds_max - (6 * (size_t)nch + 2 * kRegMaxChunks + 2 + dsl) * 8) / 8);
    // prefixes in proportion to the chunk lengths, whole wave-slots (32 G rows) when
    // they cannot all fit
    int64_t keep[kRegMaxChunks], lbase[kRegMaxChunks], tot = 0;
    for (int t = 0; t < T; ++t) tot += hlen[t];
    const int64_t align = 32 * G;
    for (int t = 0; t < T; ++t) keep[t] = tot <= cap ? hlen[t] : (cap * hlen[t] / tot) / align * align;
    if (tot > cap) {
        // the capacity the rounding left: one more wave-slot each for the chunks with the
        // most rows outside LDS (Roman, 8 chunks: 7 x 64 more rows in LDS)
        int64_t left = cap;
        for (int t = 0; t < T; ++t) left -= keep[t];
        while (left >= align) {
            int best = -1;
            for (int t = 0; t < T; ++t)
                if (keep[t] + align <= hlen[t] && (best < 0 || hlen[t] - keep[t] > hlen[best] - keep[best])) best = t;
            if (best < 0) break;
            keep[best] += align;
            left -= align;
        }
    }
    if (const char *e = getenv("GSPARSE_REG_KEEP"))
        for (int t = 0; t < T; ++t) keep[t] = std::min<int64_t>(keep[t], atoll(e));
    int64_t zs = 0;
    for (int t = 0; t < T; ++t) {
        lbase[t] = zs;
        zs += keep[t];
    }
    const uint32_t pad = (uint32_t)zs;  // the zero slot
    const size_t dyn =
        sizeof(double) * ((size_t)zs + 2 + dsl + 6 * (size_t)nch + 2 * kRegMaxChunks);
    // ELL-8 copy (uint16 p codes), overflow entries in CSR form: rebuilt only when the
    // graph, L_reg's shift or the chunk / LDS layout changed (the key)
    double regv = c->er.reg;
    int64_t regbits;
    memcpy(&regbits, &regv, sizeof(regbits));
    std::vector<int64_t> key = {c->g.epoch, regbits, n, T, G, NT, ufast ? 1 : 0, unit, dcount, dbank ? 1 : 0};
    for (int t = 0; t < T; ++t) key.insert(key.end(), {ha[t], hlen[t], keep[t]});
    auto *ocnt = (int64_t *)c->buf("er_reg_ocnt").ensure(sizeof(int64_t) * (n + 1));
    auto *optr = (int64_t *)c->buf("er_reg_optr").ensure(sizeof(int64_t) * (n + 1));
    auto *rlen = (uint16_t *)c->buf("er_reg_rlen").ensure(sizeof(uint16_t) * n);
    const bool fresh = key != c->reg_ell_key;
    if (fresh) {
        c->reg_ell_key.clear();
        c->reg_split_key.clear();
        GS_HIP(hipMemsetAsync(ocnt, 0, sizeof(int64_t) * (n + 1), s));
        k_ell8_count<<<grid_for(n, 256, 8192), 256, 0, s>>>((int32_t)n, lp, ocnt, rlen);
        exclusive_scan_i64(c, ocnt, optr, n + 1);
        GS_HIP(hipMemcpyAsync(&c->reg_nov, optr + n, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        GS_HIP(hipStreamSynchronize(s));
    }
    const int64_t nov = c->reg_nov;
    int64_t *dch;
    {
        c->reg_hch.assign(4 * kRegMaxChunks, 0);
        int64_t *hch = c->reg_hch.data();
        for (int t = 0; t < T; ++t) {
            hch[t] = ha[t];
            hch[kRegMaxChunks + t] = hlen[t];
            hch[2 * kRegMaxChunks + t] = keep[t];
            hch[3 * kRegMaxChunks + t] = lbase[t];
        }
        dch = (int64_t *)c->buf("er_reg_chunks").ensure(sizeof(int64_t) * 4 * kRegMaxChunks);
        // stream-ordered; the host table lives in the context until the next solve
        GS_HIP(hipMemcpyAsync(dch, hch, sizeof(int64_t) * 4 * kRegMaxChunks, hipMemcpyHostToDevice, s));
    }
    auto *ell = (uint4 *)c->buf("er_reg_ell").ensure(sizeof(uint4) * n);
    auto *rflag = (uint8_t *)c->buf("er_reg_rflag").ensure((size_t)n + 64);
    double *ellv = ufast ? nullptr : (double *)c->buf("er_reg_ellv").ensure(sizeof(double) * 8 * n);
    auto *ocol = (uint16_t *)c->buf("er_reg_ocol").ensure(sizeof(uint16_t) * (nov + 1));
    double *oval = ufast ? nullptr : (double *)c->buf("er_reg_oval").ensure(sizeof(double) * (nov + 1));
    if (fresh) {
        k_ell8_fill<<<grid_for(n, 256, 8192), 256, 0, s>>>(0, (int32_t)n, T, dch, pad, G,
                                                          NT == 256 ? 2 : dbank ? 3 : 1,
                                                          ufast ? (int32_t)zs + 2 : -1,
                                                          lp, li, lv, optr, ell, ellv, ocol, oval, rflag);
        GS_HIP(hipGetLastError());
        c->reg_ell_key = key;
    }
    RegArgs A{};
    // 512-thread form, whole columns: x in registers, q recomputed in the r update
    // (GSPARSE_REG_QR=1: q kept in registers from the SpMV pass, x read-modify-written
    // in Xc every iteration -- ~6x the fabric traffic for a wash in time).
    // The split form always keeps q in registers (its x lives in Xc).
    // (round 3 measured the whole-column q-in-registers form -- x read-modify-written in
    // Xc every iteration -- at parity with x in registers and 6x the fabric traffic; it
    // is no longer built, GSPARSE_REG_QR is ignored)
    A.qreg = 0;
    // Split plan: the last round of columns, when it leaves at least half the CUs idle,
    // runs as groups of P workgroups per column (k_cg_regwide<..., SPLIT>), each part a
    // contiguous range of the BLAS chunks with all its rows' p in LDS.
    // GSPARSE_REG_SPLIT=0: never; =P (>= 2): every column in P parts (tests);
    // GSPARSE_REG_SPLIT_AUTO=1: the round-5 rule, two parts per tail column when they fit.
    int ncu = 256;
    GS_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c->device));
    int P = 0;
    int64_t W = ncols;  // columns solved whole (the first W), the rest split
    split_abort_poll(c, false);
    if (c->reg_split_off && c->reg_split_off_epoch != c->g.epoch) c->reg_split_off = false;  // new graph
    if (NT == 512 && T >= 2 && ncols > 0 && !c->reg_split_off) {
        const char *se = getenv("GSPARSE_REG_SPLIT");
        const int forced = se ? atoi(se) : -1;
        if (forced >= 2) {
            P = std::min(forced, T);
            W = 0;
        } else if (forced < 0 && !getenv("GSPARSE_CG_SLOTS") && getenv("GSPARSE_REG_SPLIT_AUTO")) {
            // (round 6: off by default.  With one SpMV per iteration a whole column-iteration
            // takes ~31 us, and the last round solved whole inside the same launch -- each CU
            // starts its tail column as soon as its own columns are done -- matches or beats
            // the two-part split launch at every rank share: Roman 334 / 669 / 1,337 / 2,674
            // columns 28.6 / 44.0 / 88.1 / 164.2 ms whole vs 29.8 / 44.0 / 90.6 / 164.9 ms
            // split; profiles/r06_cg_ab/rankcols_*.  Round 3, at 44 us: 78 tail columns in 2
            // / 3 / 4 parts 13.9 / 14.5 / 30.2 ms, whole 21.8 ms.)
            const int64_t rounds = (ncols + ncu - 1) / ncu;
            const int64_t tailc = ncols - (rounds - 1) * ncu;
            if (2 * tailc <= ncu) {
                P = 2;
                W = (rounds - 1) * ncu;
            }
        }
    }
    // parts: chunk ranges as equal as possible; one geometry (G, R) for all of them
    int pc0[kRegMaxChunks + 1] = {}, Gs = 0, Rs = 0;
    size_t dyns = 0;
    if (P >= 2) {
        int tmax = 0;
        for (int h = 0, at = 0; h < P; ++h) {
            pc0[h] = at;
            at += T / P + (h < T % P ? 1 : 0);
            tmax = std::max(tmax, at - pc0[h]);
        }
        pc0[P] = T;
        int64_t plen[kRegMaxChunks];
        for (int t = 0; t < tmax; ++t) plen[t] = 0;
        for (int h = 0; h < P; ++h)
            for (int t = pc0[h]; t < pc0[h + 1]; ++t)
                plen[t - pc0[h]] = std::max<int64_t>(plen[t - pc0[h]], hlen[t]);
        const int rr = reg_geometry(512, tmax, plen, Gs);
        Rs = rr < 0 ? -1 : rr <= 16 ? 16 : rr <= 24 ? 24 : rr <= 32 ? 32 : rr <= 44 ? 44 : -1;
        for (int h = 0; h < P; ++h) {
            int64_t rows = 0;
            for (int t = pc0[h]; t < pc0[h + 1]; ++t) rows += hlen[t];
            const int th = pc0[h + 1] - pc0[h];
            dyns = std::max(dyns, sizeof(double) * ((size_t)rows + 2 + dsl + 6 * 32 * (size_t)th +
                                                    2 * kRegMaxChunks + 1));
        }
        if (Rs < 0 || Gs < 4 || dyns > lds_max) {  // does not fit: solve every column whole
            P = 0;
            W = ncols;
        }
    }
    const int64_t wslots = P ? std::min<int64_t>(ncu, std::max<int64_t>(W, 1)) : slots;
    // (-DGS_CG_XG: the second half holds each whole-column workgroup's q scratch)
    double *pg = (double *)c->buf("er_reg_pg").ensure(sizeof(double) * (GS_CG_XG ? 2 : 1) *
                                                      (size_t)std::max<int64_t>(std::max<int64_t>(wslots, slots), 1) * ldn);
    A.ld = ld;
    A.ldn = ldn;
    A.col0 = col0;
    A.ncols = W;
    A.n = (int32_t)n;
    A.Rr = Rr;
    A.Xc = Xc;
    A.pg = pg;
    A.ell = ell;
    A.ellv = ellv;
    A.optr = optr;
    A.rlen = rlen;
    A.ocol = ocol;
    A.oval = oval;
    A.diag = diag;  // L_reg's diagonal (k_l_unit), read by the whole-column unit form
    A.rflag = rflag;

    A.zslot = (int32_t)pad;
    A.maxiter = maxiter;
    A.rtol = rtol;
    A.iters = iters;
    A.T = T;
    A.ca = dch;
    A.cl = dch + kRegMaxChunks;
    A.ck = dch + 2 * kRegMaxChunks;
    A.cb = dch + 3 * kRegMaxChunks;
    A.prof = prof;
    // the whole-column launch (the first W columns); with a split tail it is issued
    // after the tail's tables and ELL are prepared, so the split launch follows it at once
    auto launch_whole = [&]() {
        if (W <= 0) return;
        if (NT == 512) {
            if (G == 1) regwide_launch_g1(A, rsel, ufast, dyn, (unsigned)wslots, s);
            else if (G == 2) regwide_launch_g2(A, rsel, ufast, dyn, (unsigned)wslots, s);
            else if (G == 4) regwide_launch_g4(A, rsel, ufast, dyn, (unsigned)wslots, s);
            else regwide_launch_g8(A, rsel, ufast, dyn, (unsigned)wslots, s);
        } else if (G == 1) regres_launch_g1(A, rsel, ufast, dyn, (unsigned)wslots, s);
        else if (G == 2) regres_launch_g2(A, rsel, ufast, dyn, (unsigned)wslots, s);
        else if (G == 4) regres_launch_g4(A, rsel, ufast, dyn, (unsigned)wslots, s);
        else regres_launch_g8(A, rsel, ufast, dyn, (unsigned)wslots, s);
        GS_HIP(hipGetLastError());
    };
    if (P < 2) {
        launch_whole();
        return;
    }

    // split tail: per-part chunk tables (LDS layout: the part's rows from slot 0, then
    // the zero slot) and an ELL whose codes each row's part resolves
    const int64_t tailn = ncols - W;
    const int64_t groups = std::min<int64_t>(tailn, ncu / P);
    int32_t hpt[kRegMaxChunks * kRegPartTab] = {};
    int64_t htab[kRegMaxChunks][4 * kRegMaxChunks] = {};
    for (int h = 0; h < P; ++h) {
        int32_t *pt = hpt + h * kRegPartTab;
        int64_t zsh = 0;
        for (int t = pc0[h]; t < pc0[h + 1]; ++t) {
            const int tl = t - pc0[h];
            pt[tl] = (int32_t)ha[t];
            pt[kRegMaxChunks + tl] = (int32_t)hlen[t];
            pt[2 * kRegMaxChunks + tl] = (int32_t)hlen[t];
            pt[3 * kRegMaxChunks + tl] = (int32_t)zsh;
            htab[h][tl] = ha[t];
            htab[h][kRegMaxChunks + tl] = hlen[t];
            htab[h][2 * kRegMaxChunks + tl] = hlen[t];
            htab[h][3 * kRegMaxChunks + tl] = zsh;
            zsh += hlen[t];
        }
        pt[4 * kRegMaxChunks] = pc0[h + 1] - pc0[h];
        pt[4 * kRegMaxChunks + 1] = (int32_t)zsh;
        pt[4 * kRegMaxChunks + 2] = pc0[h];
    }
    auto *dpt = (int32_t *)c->buf("er_reg_split_ptab").ensure(sizeof(hpt));
    auto *dtab = (int64_t *)c->buf("er_reg_split_tab").ensure(sizeof(htab));
    // stream-ordered copies from host tables the context keeps (they outlive the copies:
    // nothing below waits for the stream)
    c->reg_split_hpt.assign(hpt, hpt + sizeof(hpt) / sizeof(hpt[0]));
    c->reg_split_htab.assign(&htab[0][0], &htab[0][0] + sizeof(htab) / sizeof(int64_t));
    GS_HIP(hipMemcpyAsync(dpt, c->reg_split_hpt.data(), sizeof(hpt), hipMemcpyHostToDevice, s));
    GS_HIP(hipMemcpyAsync(dtab, c->reg_split_htab.data(), sizeof(htab), hipMemcpyHostToDevice, s));
    auto *ells = (uint4 *)c->buf("er_reg_split_ell").ensure(sizeof(uint4) * n);
    double *ellvs = ufast ? nullptr : (double *)c->buf("er_reg_split_ellv").ensure(sizeof(double) * 8 * n);
    auto *ocols = (uint16_t *)c->buf("er_reg_split_ocol").ensure(sizeof(uint16_t) * (nov + 1));
    double *ovals = ufast ? nullptr : (double *)c->buf("er_reg_split_oval").ensure(sizeof(double) * (nov + 1));
    std::vector<int64_t> skey = {P, Gs};
    skey.insert(skey.end(), pc0, pc0 + P + 1);
    const bool sfresh = skey != c->reg_split_key;
    for (int h = 0; h < P && sfresh; ++h) {
        const int32_t r0 = (int32_t)ha[pc0[h]];
        const int32_t r1 = (int32_t)(ha[pc0[h + 1] - 1] + hlen[pc0[h + 1] - 1]);
        const int32_t zsh = hpt[h * kRegPartTab + 4 * kRegMaxChunks + 1];
        k_ell8_fill<<<grid_for(r1 - r0, 256, 8192), 256, 0, s>>>(
            r0, r1, pc0[h + 1] - pc0[h], dtab + h * 4 * kRegMaxChunks, (uint32_t)zsh, Gs, 1,
            ufast ? zsh + 2 : -1, lp, li, lv, optr, ells, ellvs, ocols, ovals, nullptr);
        GS_HIP(hipGetLastError());
    }
    c->reg_split_key = skey;
    double *pgs = (double *)c->buf("er_reg_split_pg").ensure(sizeof(double) * (size_t)groups * 2 * ldn);
    double *xch = (double *)c->buf("er_reg_split_xch").ensure(sizeof(double) * (size_t)groups * 2 * kRegMaxChunks);
    auto *flg = (int32_t *)c->buf("er_reg_split_flags").ensure(sizeof(int32_t) * ((size_t)groups * P + 1));
    GS_HIP(hipMemsetAsync(flg, 0, sizeof(int32_t) * ((size_t)groups * P + 1), s));
    RegArgs B = A;
    B.col0 = col0 + W;
    B.ncols = tailn;
    B.Xc = Xc + W * ldn;
    B.pg = pgs;
    B.ell = ells;
    B.ellv = ellvs;
    B.ocol = ocols;
    B.oval = ovals;
    B.prof = nullptr;
    B.P = P;
    B.ptab = dpt;
    B.xch = xch;
    B.flags = flg;
    B.abortf = flg + (size_t)groups * P;
    // a hand-off waits at most 20 ms (a column-iteration of a split column takes
    // ~30 us; a part that is not resident never arrives)
    int wclk_khz = 100000;
    GS_HIP(hipDeviceGetAttribute(&wclk_khz, hipDeviceAttributeWallClockRate, c->device));
    B.spinmax = 20 * std::max(wclk_khz, 1);
    if (const char *e = getenv("GSPARSE_REG_SPLIT_SPIN")) B.spinmax = atoi(e);
    const unsigned grid = (unsigned)(groups * P);
    launch_whole();
    if (Gs == 4) regwide_split_launch_g4(B, Rs, ufast, dyns, grid, s);
    else regwide_split_launch_g8(B, Rs, ufast, dyns, grid, s);
    GS_HIP(hipGetLastError());
    // If the parts of a column could not all be resident at once (another process or
    // stream held CUs), the hand-offs gave up and set the abort word: the tail columns
    // are then solved again, whole, one workgroup each -- by a launch gated on that
    // word on the device (it exits at once when the split form completed), so no host
    // round trip.  The host reads the word later, without waiting (split_abort_poll),
    // counts the abort and keeps the split form off for this graph.
    RegArgs Cw = A;
    Cw.col0 = col0 + W;
    Cw.ncols = tailn;
    Cw.Xc = Xc + W * ldn;
    Cw.prof = nullptr;
    Cw.gate = B.abortf;
    const int64_t ts = std::min<int64_t>(tailn, wslots > 1 ? wslots : slots);
    if (G == 1) regwide_launch_g1(Cw, rsel, ufast, dyn, (unsigned)ts, s);
    else if (G == 2) regwide_launch_g2(Cw, rsel, ufast, dyn, (unsigned)ts, s);
    else if (G == 4) regwide_launch_g4(Cw, rsel, ufast, dyn, (unsigned)ts, s);
    else regwide_launch_g8(Cw, rsel, ufast, dyn, (unsigned)ts, s);
    GS_HIP(hipGetLastError());
    if (!c->split_abort_host) {
        GS_HIP(hipHostMalloc((void **)&c->split_abort_host, sizeof(int32_t), hipHostMallocDefault));
        GS_HIP(hipEventCreateWithFlags(&c->split_abort_ev, hipEventDisableTiming));
    }
    // the previous split launch's word must be read before its pinned slot is reused
    // (ADVICE r04): the copy may still be pending when a new launch is queued
    if (c->split_abort_pending) split_abort_poll(c, true);
    *c->split_abort_host = 0;
    GS_HIP(hipMemcpyAsync(c->split_abort_host, B.abortf, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    GS_HIP(hipEventRecord(c->split_abort_ev, s));
    c->split_abort_pending = true;
    c->split_abort_parts = P;
}

// The abort word of the last split launch, once its copy has landed (never waits unless
// `wait`): an abort turns the split form off for the graph it happened on.
void split_abort_poll(gs_ctx *c, bool wait) {
    if (!c->split_abort_pending) return;
    if (!wait && hipEventQuery(c->split_abort_ev) != hipSuccess) return;
    if (wait) GS_HIP(hipEventSynchronize(c->split_abort_ev));
    c->split_abort_pending = false;
    if (*c->split_abort_host) {
        c->reg_split_off = true;
        c->reg_split_off_epoch = c->g.epoch;
        c->split_aborts += 1;
        prof_note(c, "cg_split_abort");
        fprintf(stderr, "[gsparse] split CG hand-off timed out (%d parts); tail re-solved whole, "
                        "split form off for this graph\n", c->split_abort_parts);
    }
}

}  // namespace gs
