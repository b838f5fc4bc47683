// gs_cg_reg.hpp -- register-resident CG (ApproxER mode 5), metrics.py:284-289:
// the kernel template; instantiated per G in gs_cg_reg_g{1,2,4,8}.hip (parallel
// builds), driven by gs_cg_reg.hip.
//
// The k JL columns are independent CG solves of L_reg z = y (SciPy 1.15 cg,
// maxiter 500, rtol 1e-6) whose dot products follow OpenBLAS-SkylakeX ddot's
// order for T threads: T contiguous chunks, in each 32 FMA accumulator
// chains (chain j: rows a_t + j, a_t + j + 32, ...), then a fixed fold, a
// 16-row block and an FMA tail (gs_er.hip chunk_dot).
//
// Mode 4 (k_cg_resident) keeps a column's r, p, q, x in Infinity-Cache-
// resident slots and streams ~2 MB through each CU per column-iteration; its
// bound is the CU's memory pipeline.  Here one 512-thread workgroup per CU
// owns a column and keeps it ON the CU:
//   * r and x of every row live in registers: thread (chain, g) owns the rows
//     s = g, g + G, g + 2G, ... of its chain (G threads per chain, the rows of a
//     chain dealt round-robin), so a wave's 64 lanes touch 64 consecutive rows;
//   * p lives in LDS (a prefix of every BLAS chunk's rows, sized so the chunks
//     share the LDS in proportion; the rest in a per-workgroup global slot,
//     L2-resident, gathered under a wave-uniform branch);
//   * q is never stored: L_reg p is recomputed per row where it is needed
//     (the p.q pass and the r update), from an ELL-8 copy of L_reg with
//     uint16 columns (16 B per row, one load, shared by all CUs through L2);
//   * a dot's chain (t, j) is folded by its g = 0 lane in row order: at step u
//     it takes the G rows s = G u .. G u + G - 1 from its own and its partner
//     lanes (shuffles), so the FMA sequence is exactly OpenBLAS's;
//   * every wave finishes every dot itself (chunk fold + 16-block + tail,
//     then the chunks in order) from LDS, so the result needs no broadcast.
// Per column-iteration the memory traffic is the ELL reads (L2) and the p
// rows that do not fit LDS; everything else is LDS and registers.
#pragma once
#include <algorithm>

#include "gs_internal.hpp"

namespace gs {

static constexpr int kRegThreads = 512;                 // largest workgroup
static constexpr int kRegMaxChunks = kRegThreads / 32;  // 32 chains per chunk
// slots a thread's ELL row / p_old loads run ahead (-DGS_KPRE=: A/B variants,
// tools/variant_ab.sh)
#ifndef GS_KPRE
#define GS_KPRE 1
#endif
static constexpr int kPre = GS_KPRE;
// p_old loads of the p-update pass run this many slots ahead (-DGS_KPRE_P=)
#ifndef GS_KPRE_P
#define GS_KPRE_P GS_KPRE
#endif
static constexpr int kPreP = GS_KPRE_P;
// -DGS_CG_V2=0: the round-3 slot code of the whole-column unit form (A/B builds)
#ifndef GS_CG_V2
#define GS_CG_V2 1
#endif
// V2 p update: slots past the LDS prefix handled in groups of this many (one wait each)
#ifndef GS_PGRP
#define GS_PGRP 4
#endif
// the one-wave form (k_cg_regres, hand-pipelined gathers) keeps its own, validated
// distance: at 1 slot its results were wrong (tests m5-narrow, round 3)
static constexpr int kPreN = 4;

struct RegArgs {
    int64_t ld, ldn, col0, ncols;
    int32_t n;
    const double *Rr;     // b = Y, row-major (stride ld)
    double *Xc;           // x out: column col0 + i at Xc + i * ldn
    double *pg;           // per-workgroup p rows not held in LDS (ldn each)
    const uint4 *ell;     // [n]: the first 8 entries of each row as p codes (uint16, ascending
                          // columns; padding: zslot), see k_ell8_fill
    const double *ellv;   // [n][8] weights (weighted form), else nullptr
    const uint16_t *rlen; // [n] entries of each row of L_reg
    const int64_t *optr;  // [n+1] entries 9.. of longer rows
    const uint16_t *ocol;  // p codes
    const double *oval;

    int32_t zslot;        // LDS slot after the p rows: holds 0.0, the ELL padding code
    int32_t maxiter;
    double rtol;
    int32_t *iters;       // [k] iterations executed per column
    int32_t T;            // BLAS chunks
    const int64_t *ca, *cl;  // chunk starts / lengths (device)
    const int64_t *ck, *cb;  // rows of each chunk whose p is in LDS (a prefix), and their LDS base
    long long *prof;      // optional: workgroup 0's phase times
    int32_t qreg;         // 512-thread form: q in registers, x in Xc (see k_cg_regwide)
    // split form (k_cg_regwide<..., SPLIT>): P parts per column
    int32_t P;
    const int32_t *ptab;  // [P][kRegPartTab]: the part's chunk table, chunks, zero slot, first chunk
    double *xch;          // [groups][2][kRegMaxChunks] chunk dots by hand-off parity
    int32_t *flags;       // [groups][P] hand-off sequence numbers (zeroed before the launch)
    int32_t *abortf;      // set when a hand-off poll gave up
    int32_t spinmax;      // wait budget of one hand-off poll, in ticks of the 100 MHz
                          // constant clock (wall_clock64); 0: give up at once
    const double *diag;   // [n] L_reg's diagonal (unit form of the whole-column launch)
    const uint8_t *rflag; // [n] bit 0: a p code of the row's ELL-8 entries is global (0x8000 |
                          // row), bit 1: the row has more than 8 entries (k_ell8_fill)
    const int32_t *gate;  // optional: solve the columns only if *gate != 0 (the whole-column
                          // re-solve of a split tail whose hand-offs gave up; read once at
                          // launch, wave-uniform), else every column as usual
};
static constexpr int kRegPartTab = 4 * kRegMaxChunks + 4;

// A double held in two AGPRs.  r and x live there (read / written only through these
// asm moves, so the allocator keeps their home in the accumulation registers): with
// 256 threads a lane has 256 VGPRs + 256 AGPRs, and the VGPRs stay free for the
// slots' gathers and prefetches.
struct AgD {
    uint32_t lo, hi;
};
__device__ __forceinline__ double ag_get(const AgD &a) {
    uint32_t l, h;
    asm volatile("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3"
                 : "=v"(l), "=v"(h)
                 : "a"(a.lo), "a"(a.hi));
    return __longlong_as_double((long long)(((uint64_t)h << 32) | l));
}
__device__ __forceinline__ void ag_set(AgD &a, double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t l = (uint32_t)b, h = (uint32_t)(b >> 32);
    asm volatile("v_accvgpr_write_b32 %0, %2\n\tv_accvgpr_write_b32 %1, %3"
                 : "=a"(a.lo), "=a"(a.hi)
                 : "v"(l), "v"(h));
}

__device__ __forceinline__ double reg_uniform(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// G threads per chain (power of two), R row slots per thread, UNIT: every
// off-diagonal weight is -1.0 and every diagonal one fl((entries - 1) + 1e-6) (no
// weights loaded; q_i folds -p_j and dg * p_i); else the ELL carries the weights
template <int NT, int G, int R, bool UNIT>
__global__ void __launch_bounds__(NT) k_cg_regres(RegArgs A) {
    constexpr int CW = 64 / G;  // chains per wave
    extern __shared__ double lds[];
    const int T = A.T, nch = 32 * T;
    // LDS: p at offset 0 (a gather's address is its code * 8), the zero and scratch
    // slots, then chain sums, tail rows and the chunk table
    double *sp = lds;
    // after p: the zero slot, a scratch slot, one diagonal slot per thread, chain sums ...
    double *acc_pq = lds + A.zslot + 2 + 2 * NT, *acc_rr = acc_pq + nch;
    double *side_p = acc_pq + 2 * nch, *side_q = acc_pq + 3 * nch, *side_r = acc_pq + 4 * nch;
    double *side_x = acc_pq + 5 * nch;  // tail rows' r lives in side_r, x here
    // [4][kRegMaxChunks]: starts, lengths, LDS-resident prefix, its LDS base
    int *s_ch = reinterpret_cast<int *>(acc_pq + 6 * nch);
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < T) {
        s_ch[tid] = (int)A.ca[tid];
        s_ch[kRegMaxChunks + tid] = (int)A.cl[tid];
        s_ch[2 * kRegMaxChunks + tid] = (int)A.ck[tid];
        s_ch[3 * kRegMaxChunks + tid] = (int)A.cb[tid];
    }
    __syncthreads();
    const int jj = lane % CW, g = lane / CW;
    const int chain = (tid >> 6) * CW + jj;
    const bool live = chain < nch;
    const int t = live ? chain >> 5 : 0, j = chain & 31;
    const int L = s_ch[kRegMaxChunks + t];
    const int n32 = L & ~31;
    const int S = live ? n32 >> 5 : -1;  // chain rows; row s == S is a tail row when j < tl
    const int tl = L - n32;
    int base = s_ch[t] + j + 32 * g;  // row of slot u: base + 32 G u
    // register slots u < uc hold chain rows; the chunk's tail row s == S (j < tl) is
    // kept by the g == 0 lane with its r and x in LDS (side_r / side_x)
    int uc = S > g ? (S - g + G - 1) / G : 0;
    const bool tail = live && g == 0 && j < tl;
    const int trow = s_ch[t] + n32 + j;
    const int tix = t * 32 + j;
    int Sv = S;
    // Re-derive the per-slot rows and conditions inside every phase: left loop-
    // invariant, the compiler hoists all R of them out of the iteration loop and
    // keeps them live (hundreds of SGPRs/VGPRs, spilled to scratch).
    const int ca_t = s_ch[t], keep_t = s_ch[2 * kRegMaxChunks + t], lbase_t = s_ch[3 * kRegMaxChunks + t];
    const int zslot = A.zslot;  // LDS slot holding 0.0 (the ELL padding code)
    // explicit address spaces: a select between an LDS and a global pointer would
    // become one (slow) flat load
    typedef __attribute__((address_space(3))) double lds_f64;
    lds_f64 *spl = (lds_f64 *)sp;
    double *pgw = A.pg + (int64_t)blockIdx.x * A.ldn;
    // rows of p outside LDS: raw buffer, offsets past its size read 0 / drop the store
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(pgw, 0, (int)(A.ldn * 8), 0x00020000);
    constexpr int kOob = (int)0x80000000;
    // Loads issued under a wave-uniform branch complete inside it: left pending, the
    // join would wait vmcnt(0) on every path -- including the ELL rows in flight for the
    // next slots.  (s_waitcnt vmcnt(0), expcnt and lgkmcnt untouched: gfx9 encoding.)
    auto vm_drain = [] { __builtin_amdgcn_s_waitcnt(0x0f70); };
    if (tid == 0) spl[zslot] = 0.0;

    // p of a row lives at its code: an LDS slot (< 0x8000) or 0x8000 | row (global);
    // code_of takes a row of this lane's chunk
    auto code_of = [&](int row) {
        const int o = row - ca_t;
        return o < keep_t ? lbase_t + o : 0x8000 | row;
    };
    // LDS access always; the global one only under a wave-uniform branch (a wave's
    // rows of one slot are 32 G consecutive rows of a chunk, mostly all LDS-resident)
    auto ldc = [&](int cd) -> double {
        double v = spl[cd < 0x8000 ? cd : zslot];
        if (__builtin_amdgcn_ballot_w64(cd >= 0x8000)) {
            const double vg = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(prs, cd < 0x8000 ? kOob : (cd & 0x7fff) * 8, 0, 0));
            v = cd < 0x8000 ? v : vg;
            vm_drain();
        }
        return v;
    };
    auto stc = [&](int cd, double v) {
        spl[cd < 0x8000 ? cd : zslot + 1] = v;  // zslot + 1: a scratch slot
        if (__builtin_amdgcn_ballot_w64(cd >= 0x8000))
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), prs,
                cd < 0x8000 ? kOob : (cd & 0x7fff) * 8, 0, 0);
    };
    auto valid = [&](int u) { return u < uc; };
    // ELL rows and lengths of slot u: raw buffer loads, voffset = the lane's first row,
    // soffset = the slot's constant stride (no address arithmetic per slot).  A slot
    // past this lane's rows reads another row (or 0 past the end): never used.
    const __amdgpu_buffer_rsrc_t ers =
        __builtin_amdgcn_make_buffer_rsrc((void *)A.ell, 0, A.n * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t lrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A.rlen, 0, A.n * 2, 0x00020000);
    auto ell_row = [&](int u) -> uint4 {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(ers, base * 16, 512 * G * u, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    };
    auto len_row = [&](int u) -> int {
        return (int)__builtin_amdgcn_raw_buffer_load_b16(lrs, base * 2, 64 * G * u, 0);
    };
    auto rowof = [&](int u) { return base + 32 * G * u; };
    // own-row code of slot u: LDS slot base + off + 32 G u for the first ukeep slots,
    // else the row | 0x8000
    const int coff = lbase_t - ca_t;
    const int o0 = j + 32 * g;
    int ukeep = keep_t > o0 ? (keep_t - o0 + 32 * G - 1) / (32 * G) : 0;
    auto slot_code = [&](int u) { return rowof(u) + (u < ukeep ? coff : 0x8000); };
    auto launder = [&]() { asm volatile("" : "+v"(base), "+v"(uc), "+v"(Sv), "+v"(ukeep)); };

    // q_i = (L_reg p)_i, SciPy csr_matvec: fold from 0.0 in ascending column, products
    // rounded.  Entries are p codes.  Padding entries gather the zero slot: +-0.0 terms,
    // and acc + (+-0.0) == acc bit for bit (acc starts at +0.0 and is never -0.0).
    // Codes of global rows read past the LDS (no fault; the value is replaced under one
    // wave-uniform branch), so a slot waits for no memory load of its own and the ELL
    // rows prefetched for the next slots stay in flight.
    //
    // Unit form: every off-diagonal product is -1.0 * p_j == -p_j exactly, and the ELL
    // points the diagonal entry at this thread's diagonal slot, which holds
    // -fl(dg * p_i): the fold is acc - v over the gathered v, one subtraction per entry.
    // two diagonal slots per thread, by slot parity: a sweep issues slot u+1 (writing
    // its slot) while slot u may still read its own (a diagonal among a long row's
    // overflow entries is read when slot u folds)
    const int dslot = A.zslot + 2 + 2 * tid;
    // two halves, so a sweep can issue slot u+1's gathers before it folds slot u:
    // spmv_issue writes the diagonal slot and starts the 8 LDS gathers; spmv_fold
    // patches global entries and folds (LDS ops of one wave run in order, so the
    // diagonal slot a later spmv_issue rewrites has already been read)
    auto spmv_issue = [&](const uint4 e, int len, double pown, double (&pv)[8], int parity) {
        const uint32_t w4[4] = {e.x, e.y, e.z, e.w};
        if (UNIT) {
            const double td = ((double)(len - 1) + 1e-6) * pown;  // L_reg_ii == fl((entries - 1) + 1e-6)
            spl[dslot + parity] = -td;
        }
        // the LDS byte address of each code: one SDWA shift of its 16-bit half
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t a;
            if (k & 1)
                asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                    : "=v"(a) : "v"(w4[k >> 1]));
            else
                asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                    : "=v"(a) : "v"(w4[k >> 1]));
            pv[k] = *(lds_f64 *)(size_t)a;
        }
    };
    auto spmv_fold = [&](int row, const uint4 e, int len, double (&pv)[8]) -> double {
        const uint32_t w4[4] = {e.x, e.y, e.z, e.w};
        const bool anyg = ((w4[0] | w4[1] | w4[2] | w4[3]) & 0x80008000u) != 0;
        if (__builtin_amdgcn_ballot_w64(anyg)) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int cd = (int)((w4[k >> 1] >> (16 * (k & 1))) & 0xffffu);
                const bool gk = cd >= 0x8000;
                const double vg = __builtin_bit_cast(
                    double, __builtin_amdgcn_raw_buffer_load_b64(prs, gk ? (cd & 0x7fff) * 8 : kOob, 0, 0));
                pv[k] = gk ? vg : pv[k];
            }
            vm_drain();
        }
        double acc = 0.0;
        if (UNIT) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc = acc - pv[k];
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const double prod = A.ellv[(int64_t)row * 8 + k] * pv[k];
                acc = acc + prod;
            }
        }
        if (__builtin_amdgcn_ballot_w64(len > 8)) {  // rows longer than 8 entries: ocol / oval
            const int64_t o0 = len > 8 ? A.optr[row] : 0, o1 = len > 8 ? A.optr[row + 1] : 0;
            for (int64_t q = o0; q < o1; ++q) {
                const int cc = (int)A.ocol[q];
                const double pc = ldc(cc);
                if (UNIT) {
                    acc = acc - pc;
                } else {
                    const double prod = A.oval[q] * pc;
                    acc = acc + prod;
                }
            }
            vm_drain();
        }
        return acc;
    };
    auto spmv = [&](int row, const uint4 e, int len, double pown) -> double {
        double pv[8];
        spmv_issue(e, len, pown, pv, 0);  // tail rows: parity 0, issued and folded alone
        return spmv_fold(row, e, len, pv);
    };

    // one step of every chain: rows s = G u + gg (gg < G) in order, folded by the g = 0 lane
    auto chain_step = [&](double &acc, double av, double bv, int u) {
        double as[G], bs[G];
        as[0] = av;  // the folding lane's own row (g = 0)
        bs[0] = bv;
#pragma unroll
        for (int gg = 1; gg < G; ++gg) {
            as[gg] = __shfl(av, jj + CW * gg, 64);
            bs[gg] = __shfl(bv, jj + CW * gg, 64);
        }
#pragma unroll
        for (int gg = 0; gg < G; ++gg)
            if (G * u + gg < Sv) acc = __builtin_fma(as[gg], bs[gg], acc);
        // fold now: deferred, every slot's shuffled operands would stay live to the end
        asm volatile("" : "+v"(acc));
    };

    // OpenBLAS finish of one dot (every wave computes it; lane = chunk)
    auto finish = [&](const double *acc32all, const double *xa_all, const double *xb_all) -> double {
        double d = 0.0;
        if (lane < T) {
            const int Lt = s_ch[kRegMaxChunks + lane];
            const int n1 = Lt & ~15, n32t = n1 & ~31;
            const double *a32 = acc32all + lane * 32;
            const double *xa = xa_all + lane * 32, *xb = xb_all + lane * 32;
            double dot = 0.0;
            if (n1) {
                // b[4q + l] = acc[8q + l] + acc[8q + 4 + l] (+ the 16-block row 4q + l),
                // c4[l] = ((b[l] + b[4 + l]) + b[8 + l]) + b[12 + l] -- one l at a time
                const bool blk = n1 > n32t;
                double c4[4];
                for (int l = 0; l < 4; ++l) {
                    double cl = 0.0;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        double b = a32[8 * q + l] + a32[8 * q + 4 + l];
                        if (blk) b = __builtin_fma(xa[4 * q + l], xb[4 * q + l], b);
                        cl = q == 0 ? b : cl + b;
                    }
                    c4[l] = cl;
                }
                dot = (c4[0] + c4[2]) + (c4[1] + c4[3]);
            }
            for (int i = 0; i < 15; ++i)
                if (n1 + i < Lt) {
                    const int ix = n1 - n32t + i;
                    dot = __builtin_fma(xb[ix], xa[ix], dot);
                }
            d = dot;
        }
        if (T == 1) return reg_uniform(__shfl(d, 0, 64));
        double total = 0.0;
        for (int tt = 0; tt < T; ++tt) total = total + __shfl(d, tt, 64);
        return reg_uniform(total);
    };

    long long tp[5] = {0, 0, 0, 0, 0};
    long long tmark = wall_clock64();
    auto lap = [&](int ph) {
        const long long tn = wall_clock64();
        tp[ph] += tn - tmark;
        tmark = tn;
    };

    const int64_t ncols = (A.gate && *A.gate == 0) ? 0 : A.ncols;
    for (int64_t ci = blockIdx.x; ci < ncols; ci += gridDim.x) {
        const int64_t c = A.col0 + ci;
        AgD r[R], x[R];
        // r = b.copy(); rho_0 = b.b
        {
            launder();
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                ag_set(x[u], 0.0);
                const double b = valid(u) ? A.Rr[(int64_t)rowof(u) * A.ld + c] : 0.0;
                ag_set(r[u], b);
                chain_step(acc, b, b, u);
            }
            if (g == 0 && live) acc_rr[chain] = acc;
            if (tail) {
                side_r[tix] = A.Rr[(int64_t)trow * A.ld + c];
                side_x[tix] = 0.0;
            }
        }
        __syncthreads();
        double rr = finish(acc_rr, side_r, side_r);
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
            // p = beta p + r (two roundings); x += alpha_{it-1} p_{it-1} rides along
            launder();
            if (it == 0) {
#pragma unroll
                for (int u = 0; u < R; ++u)
                    if (valid(u)) stc(slot_code(u), ag_get(r[u]));
            } else {
                // four slots at a time: their p_old loads in flight together; LDS-only
                // groups (the common case) skip the global path under a uniform branch
                static_assert(R % 4 == 0, "row slots come in groups of four");
#pragma unroll
                for (int u0 = 0; u0 < R; u0 += 4) {
                    int cdv[4];
                    bool glob = false;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        cdv[i] = valid(u0 + i) ? slot_code(u0 + i) : zslot + 1;
                        glob = glob || cdv[i] >= 0x8000;
                    }
                    const bool wg = __builtin_amdgcn_ballot_w64(glob) != 0;
                    double po[4], pn[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) po[i] = wg ? ldc(cdv[i]) : spl[cdv[i]];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const double t1 = alpha_prev * po[i];
                        ag_set(x[u0 + i], ag_get(x[u0 + i]) + t1);
                        const double pb = po[i] * beta;
                        pn[i] = pb + ag_get(r[u0 + i]);
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        if (wg) stc(cdv[i], pn[i]);
                        else spl[cdv[i]] = pn[i];  // invalid slots write the scratch slot
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (tail) {
                if (it == 0) {
                    stc(code_of(trow), side_r[tix]);
                } else {
                    const double po = ldc(code_of(trow));
                    const double t1 = alpha_prev * po;
                    side_x[tix] = side_x[tix] + t1;
                    const double pb = po * beta;
                    stc(code_of(trow), pb + side_r[tix]);
                }
            }
            __syncthreads();
            lap(0);
            // q = L_reg p and the chains of p.q
            {
                launder();
                double acc = 0.0;
                uint4 eb[R];  // ELL rows and lengths, kPreN slots ahead
                int lb[R];
                double pw[R];     // own p, two slots ahead
                double pg[R][8];  // gathers, one slot ahead
#pragma unroll
                for (int u = 0; u < kPreN && u < R; ++u) {
                    eb[u] = ell_row(u);
                    lb[u] = len_row(u);
                }
                pw[0] = valid(0) ? ldc(slot_code(0)) : 0.0;
                if (R > 1) pw[1] = valid(1) ? ldc(slot_code(1)) : 0.0;
                spmv_issue(eb[0], lb[0], pw[0], pg[0], 0);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPreN < R) {
                        eb[u + kPreN] = ell_row(u + kPreN);
                        lb[u + kPreN] = len_row(u + kPreN);
                    }
                    if (u + 2 < R) pw[u + 2] = valid(u + 2) ? ldc(slot_code(u + 2)) : 0.0;
                    if (u + 1 < R) spmv_issue(eb[u + 1], lb[u + 1], pw[u + 1], pg[u + 1], (u + 1) & 1);
                    double qv = 0.0;
                    if (valid(u)) qv = spmv_fold(rowof(u), eb[u], lb[u], pg[u]);
                    chain_step(acc, pw[u], qv, u);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_pq[chain] = acc;
                if (tail) {
                    const double pt = ldc(code_of(trow));
                    side_q[tix] = spmv(trow, A.ell[trow], (int)A.rlen[trow], pt);
                    side_p[tix] = pt;
                }
            }
            __syncthreads();
            lap(1);
            const double pq = finish(acc_pq, side_p, side_q);
            const double alpha = rho_cur / pq;
            lap(2);
            // r -= alpha q (q recomputed), chains of r.r
            {
                launder();
                double acc = 0.0;
                uint4 eb[R];
                int lb[R];
                double pw[R];
                double pg[R][8];
#pragma unroll
                for (int u = 0; u < kPreN && u < R; ++u) {
                    eb[u] = ell_row(u);
                    lb[u] = len_row(u);
                }
                pw[0] = (UNIT && valid(0)) ? ldc(slot_code(0)) : 0.0;
                if (R > 1) pw[1] = (UNIT && valid(1)) ? ldc(slot_code(1)) : 0.0;
                spmv_issue(eb[0], lb[0], pw[0], pg[0], 0);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPreN < R) {
                        eb[u + kPreN] = ell_row(u + kPreN);
                        lb[u + kPreN] = len_row(u + kPreN);
                    }
                    if (u + 2 < R) pw[u + 2] = (UNIT && valid(u + 2)) ? ldc(slot_code(u + 2)) : 0.0;
                    if (u + 1 < R) spmv_issue(eb[u + 1], lb[u + 1], pw[u + 1], pg[u + 1], (u + 1) & 1);
                    double rn = 0.0;
                    if (valid(u)) {
                        const double t2 = alpha * spmv_fold(rowof(u), eb[u], lb[u], pg[u]);
                        rn = ag_get(r[u]) - t2;
                        ag_set(r[u], rn);
                    }
                    chain_step(acc, rn, rn, u);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_rr[chain] = acc;
                if (tail) {
                    const double pt = UNIT ? ldc(code_of(trow)) : 0.0;
                    const double t2 = alpha * spmv(trow, A.ell[trow], (int)A.rlen[trow], pt);
                    side_r[tix] = side_r[tix] - t2;
                }
            }
            __syncthreads();
            lap(3);
            rr = finish(acc_rr, side_r, side_r);
            rho_prev = rho_cur;
            alpha_prev = alpha;
            done = it + 1;
        }
        // x: b (||b|| == 0), 0 (no iteration), or the last pending update
        launder();
        double *xo = A.Xc + ci * A.ldn;
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (valid(u)) {
                const int row = rowof(u);
                double v;
                if (bn == 0.0) v = ag_get(r[u]);
                else if (done == 0) v = 0.0;
                else {
                    const double t1 = alpha_prev * ldc(slot_code(u));
                    v = (done > 1 ? ag_get(x[u]) : 0.0) + t1;
                }
                xo[row] = v;
            }
        if (tail) {
            double v;
            if (bn == 0.0) v = side_r[tix];
            else if (done == 0) v = 0.0;
            else {
                const double t1 = alpha_prev * ldc(code_of(trow));
                v = (done > 1 ? side_x[tix] : 0.0) + t1;
            }
            xo[trow] = v;
        }
        if (tid == 0) A.iters[c] = done;
        __syncthreads();  // the next column's b.b chains reuse acc_rr / side_r
    }
    if (A.prof && blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < 5; ++i) A.prof[i] = tp[i];
}


// one launch of k_cg_regres<256, G, R, UNIT> (defined in gs_cg_reg_g<G>.hip)
#define GS_REGRES_LAUNCH_DECL(G_)                                                            \
    void regres_launch_g##G_(const RegArgs &A, int R, bool unit, size_t dyn, unsigned slots, \
                             hipStream_t s);
GS_REGRES_LAUNCH_DECL(1)
GS_REGRES_LAUNCH_DECL(2)
GS_REGRES_LAUNCH_DECL(4)
GS_REGRES_LAUNCH_DECL(8)
#undef GS_REGRES_LAUNCH_DECL
// one launch of k_cg_regwide<G, R, UNIT> (512 threads, gs_cg_wide.hpp)
#define GS_REGWIDE_LAUNCH_DECL(G_)                                                            \
    void regwide_launch_g##G_(const RegArgs &A, int R, bool unit, size_t dyn, unsigned slots, \
                              hipStream_t s);
GS_REGWIDE_LAUNCH_DECL(1)
GS_REGWIDE_LAUNCH_DECL(2)
GS_REGWIDE_LAUNCH_DECL(4)
GS_REGWIDE_LAUNCH_DECL(8)
#undef GS_REGWIDE_LAUNCH_DECL
// split form, 4 or 8 threads per chain (gs_cg_reg_s4.hip, gs_cg_reg_s8.hip)
void regwide_split_launch_g4(const RegArgs &A, int R, bool unit, size_t dyn, unsigned grid, hipStream_t s);
void regwide_split_launch_g8(const RegArgs &A, int R, bool unit, size_t dyn, unsigned grid, hipStream_t s);

// one launch of the kernel: R row slots (24 / 48 / 64 / 88), unit or weighted form
#define GS_REGRES_LAUNCH_DEF(G_)                                                              \
    void regres_launch_g##G_(const RegArgs &A, int R, bool unit, size_t dyn, unsigned slots,  \
                             hipStream_t s) {                                                 \
        auto go = [&](auto kern) {                                                            \
            GS_HIP(hipFuncSetAttribute((const void *)kern,                                    \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn)); \
            kern<<<slots, 256, dyn, s>>>(A);                                                  \
        };                                                                                    \
        if (unit) {                                                                           \
            if (R == 24) go(k_cg_regres<256, G_, 24, true>);                                 \
            else if (R == 48) go(k_cg_regres<256, G_, 48, true>);                            \
            else if (R == 64) go(k_cg_regres<256, G_, 64, true>);                            \
            else go(k_cg_regres<256, G_, 88, true>);                                         \
        } else {                                                                              \
            if (R == 24) go(k_cg_regres<256, G_, 24, false>);                                \
            else if (R == 48) go(k_cg_regres<256, G_, 48, false>);                           \
            else if (R == 64) go(k_cg_regres<256, G_, 64, false>);                           \
            else go(k_cg_regres<256, G_, 88, false>);                                        \
        }                                                                                     \
    }

}  // namespace gs
