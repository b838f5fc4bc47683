// gs_cg_wide.hpp -- the 512-thread form of the register-resident CG (ApproxER mode
// 5; design notes in gs_cg_reg.hpp).  Two waves per SIMD, 256 registers per lane:
// r and x of up to 44 row slots per thread, the allocator's own VGPR / AGPR split.
// The second wave on each SIMD hides the LDS and fp64 latencies that the
// one-wave form (k_cg_regres, up to 88 slots) must pipeline by hand, so this
// form runs wherever the slots fit 44 (Roman-empire: 8 chunks, 2 threads per
// chain, 44 slots); k_cg_regres takes the larger graphs.  Instantiated per G in
// gs_cg_reg_g{1,2,4,8}.hip.
#pragma once
#include "gs_cg_reg.hpp"

// GS_CG_QS (default 1): whole columns (x in registers) store q = L_reg p of the SpMV pass
// in the column's own Xc output column (Infinity Cache scratch until x is written there at
// the end), and the r update reads it back (GS_CG_QPRE slots ahead) instead of
// recomputing the SpMV: one SpMV per iteration, the same arithmetic.  Roman, T = 8: r
// update 15.8 -> 5.9 us per column-iteration, 210.7 -> 167.6 ms per step (-DGS_CG_QS=0:
// the round-5 form; profiles/r06_cg_ab/)
#ifndef GS_CG_QS
#define GS_CG_QS 1
#endif
// (Roman, T = 8: q read 8 slots ahead 167.6 ms per step, 4 ahead 173.7, 12 ahead 168.1;
// profiles/r06_cg_ab/)
#ifndef GS_CG_QPRE
#define GS_CG_QPRE 8
#endif
// cache policy bits of the q stores / loads: 2 = nt (streaming).  The 256 CUs' q columns
// (46 MB) evict the ELL rows, diagonals and global p rows the SpMV gathers from the XCDs'
// L2 with the default policy: 189.9 ms per step, 173.7 with nt (profiles/r06_cg_ab/)
#ifndef GS_CG_QAUX
#define GS_CG_QAUX 2
#endif
// cache policy bits of the split tail's x read-modify-write in Xc (q-in-registers form)
#ifndef GS_CG_XAUX
#define GS_CG_XAUX 0
#endif
// -DGS_CG_XG=1 (A/B): whole columns keep x in their Xc column instead of registers (88
// VGPRs freed at 44 slots), q in a per-workgroup scratch (the second half of A.pg); the r
// update reads q, x and the global p rows GS_CG_QPRE slots ahead and writes x
#ifndef GS_CG_XG
#define GS_CG_XG 0
#endif

namespace gs {

// byte address (p code * 8) of the low / high 16-bit p code of an ELL word: one SDWA
// shift (word select + shift) instead of an extract and a shift
template <int HI>
__device__ __forceinline__ uint32_t wide_code_addr(uint32_t w) {
    uint32_t a;
    if (HI)
        asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
            : "=v"(a) : "v"(w));
    else
        asm("v_lshlrev_b32_sdwa %0, 3, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
            : "=v"(a) : "v"(w));
    return a;
}

// v of lane K of each quad (DPP quad_perm broadcast, both dwords)
template <int K>
__device__ __forceinline__ double wide_quad_bcast(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)b, K * 0x55, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), K * 0x55, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// v of lane ln (wave-uniform ln), as a scalar
__device__ __forceinline__ double wide_readlane(double v, int ln) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, ln);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), ln);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// G threads per chain (power of two), R row slots per thread, UNIT: every
// off-diagonal weight is -1.0 and every diagonal one fl((entries - 1) + 1e-6) (no
// weights loaded; q_i folds -p_j and dg * p_i); else the ELL carries the weights.
// QR: q of the slots stays in the registers x used to hold, from the SpMV pass to the
// r update (one SpMV per iteration instead of two); x lives in its output column of
// Xc (L2 / Infinity Cache) and is updated there in the r-update pass, x += alpha p
// in SciPy's own (non-deferred) order.
// SPLIT: a column is solved by a group of A.P workgroups (parts), part h owning a
// contiguous range of the BLAS chunks (all its rows' p in LDS).  Every part publishes
// its rows' p (write-through sc1 stores, buffer by iteration parity) for the other
// parts' SpMV, and its chunk dots (buffer by hand-off parity); three flag hand-offs per
// iteration (after the p update, before each dot's chunk sum) -- MI355X_MICROARCH.md's
// drained-sc1 recipe: sc1 payload, s_waitcnt vmcnt(0), barrier, one sc1 flag store, sc1
// polls.  The chunk dots are added in global chunk order, so the bits are those of
// the one-workgroup solve.  Used for the last, partly occupied round of columns.
template <int G, int R, bool UNIT, bool QR, bool SPLIT = false>
__global__ void __launch_bounds__(kRegThreads) k_cg_regwide(RegArgs A) {
    constexpr int CW = 64 / G;  // chains per wave
    // V2 (whole columns, unit weights): each slot's "any p code global" and "any row
    // longer than 8" tests are bits of two wave-uniform masks built once per launch (one
    // scalar bit test per slot instead of a vector OR / compare / ballot), and the
    // diagonal entry is loaded from L_reg's diagonal (one 8-B load instead of the entry
    // count's load, convert and add) -- the same bits as the count-derived value, which
    // is checked equal at setup for the unit form
    constexpr bool V2 = GS_CG_V2 && UNIT && !SPLIT;
    // V2, two threads per chain: each lane's diagonal slot in the bank after its own p
    // rows' bank (see dslot below)
    constexpr bool DBANK = V2 && G == 2;
    // q of the SpMV pass kept for the r update in the column's Xc column (GS_CG_QS)
    constexpr bool QS = GS_CG_QS && !QR && !SPLIT;
    // (GS_CG_XG) whole columns in the x-in-Xc form with q stored, not kept in registers
    constexpr bool QSX = GS_CG_XG && QR && !SPLIT;
    extern __shared__ double lds[];
    const int part = SPLIT ? (int)(blockIdx.x % (unsigned)A.P) : 0;
    const int group = SPLIT ? (int)(blockIdx.x / (unsigned)A.P) : (int)blockIdx.x;
    const int ngroups = SPLIT ? (int)(gridDim.x / (unsigned)A.P) : (int)gridDim.x;
    // SPLIT: this part's chunk table, [4][kRegMaxChunks] then chunks, zero slot, first chunk
    const int32_t *ptab = SPLIT ? A.ptab + part * kRegPartTab : nullptr;
    const int T = SPLIT ? ptab[4 * kRegMaxChunks] : A.T, nch = 32 * T;
    const int zslot = SPLIT ? ptab[4 * kRegMaxChunks + 1] : A.zslot;  // LDS slot holding 0.0
    const int t0g = SPLIT ? ptab[4 * kRegMaxChunks + 2] : 0;          // global index of chunk 0
    const int Tg = SPLIT ? A.T : T;                                    // chunks of the whole column
    // LDS: p at offset 0 (a gather's address is its code * 8), the zero and scratch
    // slots, (unit form) one diagonal slot per thread, then chain sums, tail rows and
    // the chunk table
    double *sp = lds;
    double *acc_pq = lds + zslot + 2 + (UNIT ? kRegThreads : 0), *acc_rr = acc_pq + nch;
    double *side_p = acc_pq + 2 * nch, *side_q = acc_pq + 3 * nch, *side_r = acc_pq + 4 * nch;
    double *side_x = acc_pq + 5 * nch;  // tail rows' r lives in side_r, x here
    // [4][kRegMaxChunks]: starts, lengths, LDS-resident prefix, its LDS base (SPLIT: then
    // the hand-off verdict word)
    int *s_ch = reinterpret_cast<int *>(acc_pq + 6 * nch);
    const int tid = threadIdx.x, lane = tid & 63;
    if (tid < T) {
        if constexpr (SPLIT) {
            for (int k4 = 0; k4 < 4; ++k4) s_ch[k4 * kRegMaxChunks + tid] = ptab[k4 * kRegMaxChunks + tid];
        } else {
            s_ch[tid] = (int)A.ca[tid];
            s_ch[kRegMaxChunks + tid] = (int)A.cl[tid];
            s_ch[2 * kRegMaxChunks + tid] = (int)A.ck[tid];
            s_ch[3 * kRegMaxChunks + tid] = (int)A.cb[tid];
        }
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
    // Re-derive the per-slot rows and conditions inside every phase: left loop-
    // invariant, the compiler hoists all R of them out of the iteration loop and
    // keeps them live (hundreds of SGPRs/VGPRs, spilled to scratch).
    int ulds = 0;  // set below
    uint64_t gmask = 0, lmask = 0;  // V2 slot masks, set below
    auto launder = [&]() {
        asm volatile("" : "+v"(base), "+v"(uc), "+s"(ulds));
        if constexpr (V2) asm volatile("" : "+s"(gmask), "+s"(lmask));
    };
    const int ca_t = s_ch[t], keep_t = s_ch[2 * kRegMaxChunks + t], lbase_t = s_ch[3 * kRegMaxChunks + t];
    // slots u < ulds hold LDS-resident rows in every lane of the wave (a slot's rows are
    // 32 G consecutive rows of one chunk per lane group and the prefixes are whole
    // multiples of 32 G, so this is the wave's common prefix): their p lives at the
    // byte address lds0 + 256 G u, an immediate offset -- no per-slot code, compare
    // or select, and no global fix-up branch
    {
        int uk = R;  // lanes without chain rows never limit it
        if (live) {
            const int o0 = base - ca_t;
            uk = keep_t > o0 ? (keep_t - o0 + 32 * G - 1) / (32 * G) : 0;
        }
        for (int off = 32; off >= 1; off >>= 1) uk = min(uk, __shfl_xor(uk, off, 64));
        ulds = __builtin_amdgcn_readfirstlane(uk);
    }
    auto lds0 = [&]() -> uint32_t { return (uint32_t)(lbase_t + base - ca_t) * 8u; };
    // explicit address spaces: a select between an LDS and a global pointer would
    // become one (slow) flat load
    typedef __attribute__((address_space(3))) double lds_f64;
    auto lds_at = [](uint32_t a) -> double { return *(lds_f64 *)(uintptr_t)a; };
    auto lds_put = [](uint32_t a, double v) { *(lds_f64 *)(uintptr_t)a = v; };
    lds_f64 *spl = (lds_f64 *)sp;
    // rows of p outside LDS: raw buffer, offsets past its size read 0 / drop the store.
    // SPLIT: the group's published p (two iteration-parity halves, poff selects one;
    // sc1 loads and stores, so no CU's L1 serves a stale line)
    double *pgw = A.pg + (int64_t)group * (SPLIT ? 2 : 1) * A.ldn;
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(pgw, 0, (int)(A.ldn * 8 * (SPLIT ? 2 : 1)), 0x00020000);
    constexpr int kOob = (int)0x80000000;
    constexpr int kAux = SPLIT ? 16 : 0;  // cache policy of the global p accesses (16: sc1)
    int poff = 0;                          // SPLIT: byte offset of this iteration's p half
    // s_waitcnt vmcnt(0) inside a branch that loads p from the global slot: the waitcnt
    // pass then sees no pending load at the join, and the ELL rows prefetched for the
    // next slots stay in flight (otherwise every slot waits for them: vmcnt(0))
    auto vm_drain = [] { __builtin_amdgcn_s_waitcnt(0x0f70); };
    // ELL rows and entry counts: raw buffers (row offset in a VGPR, the slot's 32 G u
    // rows as a scalar offset; rows past n read 0 and belong to no valid slot)
    const __amdgpu_buffer_rsrc_t ers =
        __builtin_amdgcn_make_buffer_rsrc((void *)A.ell, 0, (int)(A.n * 16), 0x00020000);
    const __amdgpu_buffer_rsrc_t lrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)A.rlen, 0, (int)(A.n * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(V2 ? A.diag : nullptr), 0, (int)(V2 ? A.n * 8 : 0),
                                          0x00020000);
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
                double, __builtin_amdgcn_raw_buffer_load_b64(prs, cd < 0x8000 ? kOob : (cd & 0x7fff) * 8 + poff, 0, kAux));
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
                cd < 0x8000 ? kOob : (cd & 0x7fff) * 8 + poff, 0, kAux);
    };
    // SPLIT: publish p of an own row (kept in LDS) for the other parts
    auto publish = [&](int row, double v) {
        if constexpr (SPLIT)
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), prs, row * 8 + poff, 0, 16);
    };
    auto valid = [&](int u) { return u < uc; };
    auto ell_row = [&](int u) -> uint4 {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(ers, base * 16, 512 * G * u, 0);
        return make_uint4(v[0], v[1], v[2], v[3]);
    };
    auto len_row = [&](int u) -> int {
        return (int)__builtin_amdgcn_raw_buffer_load_b16(lrs, base * 2, 64 * G * u, 0);
    };
    auto diag_row = [&](int u) -> double {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(drs, base * 8, 256 * G * u, 0));
    };
    auto rowof = [&](int u) { return base + 32 * G * u; };
    // V2: bit u of gmask / lmask = some lane of this wave has a global p code / a row
    // longer than 8 entries in slot u (rows of invalid slots contribute nothing)
    // (laundered with the slot geometry: hoisted, their R bit tests would stay live as
    // 2 R booleans across the iteration loop)
    if constexpr (V2) {
        // one slot at a time (once per launch): the loads of all slots in flight would keep
        // 2 R ballots live at once
        for (int u = 0; u < R; ++u) {
            asm volatile("" : "+s"(gmask), "+s"(lmask));
            const int f = u < uc ? (int)A.rflag[base + 32 * G * u] : 0;
            if (__builtin_amdgcn_ballot_w64((f & 1) != 0)) gmask |= 1ull << u;
            if (__builtin_amdgcn_ballot_w64((f & 2) != 0)) lmask |= 1ull << u;
        }
    }

    // q_i = (L_reg p)_i, SciPy csr_matvec: fold from 0.0 in ascending column, products
    // rounded; pown receives p_i.  Entries are p codes.  Unit form: off-diagonal
    // products are -p_j exactly (-1.0 * x == -x) and the diagonal one td = fl(dg * p_i);
    // the diagonal entry's code is this thread's diagonal slot, which receives -td
    // before the gathers (a wave's LDS operations complete in order), so every entry
    // folds as acc - v: acc - (-td) == acc + td and acc - p_j == acc + (-p_j) bit for bit.
    // Padding entries gather the zero slot: +-0.0 terms, and acc + (+-0.0) == acc bit
    // for bit (acc starts at +0.0 and is never -0.0).  Codes of global rows read past
    // the LDS (no fault; the value is replaced under one wave-uniform branch), so the
    // slot issues no memory load whose result it waits for -- the ELL rows prefetched
    // for the next slots stay in flight.
    // (DBANK) each 32-lane group's slots stay the 32 after zslot + 2 + (tid & ~31), permuted
    // so lane l's sits in bank (own p bank + 1) mod 32 -- own rows lbase_t + l + 64 u --
    // and the diagonal reads of a gather collide less with the p reads of lanes whose
    // entries are shifted by a lower chord (tools/lds_bank_sim.py: the gathers' extra LDS
    // cycles on the Roman layout 40 % -> 35 % over conflict-free); k_ell8_fill (dmul 3)
    // gives the diagonal entries the same codes
    const int dslot0 = zslot + 2 + (tid & ~31);
    const int dslot = DBANK ? dslot0 + ((lbase_t + (tid & 31) + 1 - dslot0) & 31) : zslot + 2 + tid;
    // u >= 0: register slot u (LDS fast path when u < ulds); u < 0: a tail row
    auto spmv = [&](int row, const uint4 e, int len, double &pown, int u) -> double {
        const bool fast = u >= 0 && u < ulds;  // wave-uniform
        const int self = fast ? 0 : code_of(row);
        const uint32_t w4[4] = {e.x, e.y, e.z, e.w};
        uint32_t ad[8];  // LDS byte addresses; global codes land past the LDS (read as 0)
#pragma unroll
        for (int k = 0; k < 8; ++k) ad[k] = (k & 1) ? wide_code_addr<1>(w4[k >> 1]) : wide_code_addr<0>(w4[k >> 1]);
        double td = 0.0;
        if (UNIT) {
            pown = fast ? lds_at(lds0() + 256u * G * u) : ldc(self);
            const double dg = (double)(len - 1) + 1e-6;  // UNIT: L_reg_ii == fl((entries - 1) + 1e-6)
            td = dg * pown;
            spl[dslot] = -td;
        }
        double pv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) pv[k] = lds_at(ad[k]);
        if (!UNIT) pown = fast ? lds_at(lds0() + 256u * G * u) : spl[self];
        const bool anyg = ((w4[0] | w4[1] | w4[2] | w4[3]) & 0x80008000u) != 0 || (!UNIT && !fast && self >= 0x8000);
        if (__builtin_amdgcn_ballot_w64(anyg)) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool gk = ad[k] >= 0x8000u * 8;
                const double vg = __builtin_bit_cast(
                    double, __builtin_amdgcn_raw_buffer_load_b64(prs, gk ? (int)(ad[k] & 0x3fff8u) + poff : kOob, 0, kAux));
                pv[k] = gk ? vg : pv[k];
            }
            if (!UNIT && !fast) pown = ldc(self);
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
                if (UNIT) acc = acc - pc;  // the diagonal's code is the diagonal slot
                else acc = acc + A.oval[q] * pc;
            }
            vm_drain();
        }
        return acc;
    };

    // V2 slot u (u >= 0): dg = L_reg_ii loaded, the global fix-up and the long-row tail
    // under the slot's mask bits; the arithmetic is spmv()'s, operation for operation
    auto spmv2 = [&](int row, const uint4 e, double dg, double &pown, int u) -> double {
        const bool fast = u < ulds;  // wave-uniform
        const int self = fast ? 0 : code_of(row);
        const uint32_t w4[4] = {e.x, e.y, e.z, e.w};
        uint32_t ad[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) ad[k] = (k & 1) ? wide_code_addr<1>(w4[k >> 1]) : wide_code_addr<0>(w4[k >> 1]);
        pown = fast ? lds_at(lds0() + 256u * G * u) : ldc(self);
        const double td = dg * pown;
        spl[dslot] = -td;
        double pv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) pv[k] = lds_at(ad[k]);
        uint64_t gm = gmask;  // tested here, not hoisted (see launder)
        asm volatile("" : "+s"(gm));
        if ((gm >> u) & 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool gk = ad[k] >= 0x8000u * 8;
                const double vg = __builtin_bit_cast(
                    double, __builtin_amdgcn_raw_buffer_load_b64(prs, gk ? (int)(ad[k] & 0x3fff8u) + poff : kOob, 0, kAux));
                pv[k] = gk ? vg : pv[k];
            }
            vm_drain();
        }
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) acc = acc - pv[k];
        uint64_t lm = lmask;
        asm volatile("" : "+s"(lm));
        if ((lm >> u) & 1) {  // rows longer than 8 entries: ocol
            const int64_t o0 = A.optr[row], o1 = A.optr[row + 1];
            for (int64_t q = o0; q < o1; ++q) acc = acc - ldc((int)A.ocol[q]);
            vm_drain();
        }
        return acc;
    };

    // lanes 0..31 receive v of lanes 32..63 (v_permlane32_swap)
    auto upper_half = [](double v) -> double {
        const uint64_t b = (uint64_t)__double_as_longlong(v);
        const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
        const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
        return __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
    };
    // one step of every chain: rows s = G u + gg (gg < G) in order, folded by the g = 0 lane
    auto chain_step = [&](double &acc, double av, double bv, int u, bool same = false) {
        double as[G], bs[G];
        as[0] = av;  // the folding lane's own row (g = 0)
        bs[0] = bv;
        if (G == 2 && V2) {
            // one swap per dword of (v, v): the returned vdst keeps the own value in lanes
            // 0..31, the returned src holds lanes 32..63's there -- v is dead afterwards, so
            // one copy per dword instead of two
            auto sw = [](double v, double &own, double &part) {
                const uint64_t b = (uint64_t)__double_as_longlong(v);
                const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)b, (uint32_t)b, false, false);
                const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(b >> 32), (uint32_t)(b >> 32), false, false);
                own = __longlong_as_double((long long)(((uint64_t)hi[0] << 32) | lo[0]));
                part = __longlong_as_double((long long)(((uint64_t)hi[1] << 32) | lo[1]));
            };
            sw(av, as[0], as[G - 1]);
            if (same) {
                bs[0] = as[0];
                bs[G - 1] = as[G - 1];
            } else {
                sw(bv, bs[0], bs[G - 1]);
            }
        } else if (G == 2) {  // partner = lane + 32: one permlane swap per dword, no LDS
            as[G - 1] = upper_half(av);
            bs[G - 1] = same ? as[G - 1] : upper_half(bv);  // same: bv is av
        } else {
#pragma unroll
            for (int gg = 1; gg < G; ++gg) {
                as[gg] = __shfl(av, jj + CW * gg, 64);
                bs[gg] = __shfl(bv, jj + CW * gg, 64);
            }
        }
        // rows past the chain's end hold exact zeros (unset p / q, r of invalid slots):
        // fma(0, 0, acc) == acc, acc never being -0.0 -- no per-row test
#pragma unroll
        for (int gg = 0; gg < G; ++gg) acc = __builtin_fma(as[gg], bs[gg], acc);
        // fold now: deferred, every slot's shuffled operands would stay live to the end
        asm volatile("" : "+v"(acc));
    };

    // SPLIT hand-off: every wave drains its (sc1) stores, then one lane raises this
    // part's flag to the next sequence number and polls the group's other flags.  A
    // poll that never matches (a part that cannot arrive) gives up after A.spinmax
    // ticks of the constant clock (20 ms by default) and sets the abort word: from then on this workgroup's hand-offs are barriers
    // only, so the launch runs out (its results are discarded, the host reports the
    // abort) instead of hanging the GPU.  (No early return: a divergent exit from the
    // column loop breaks the uniform-register allocation of this kernel.)
    int32_t hseq = 0;
    bool bad = false;
    int32_t *gflags = SPLIT ? A.flags + (int64_t)group * A.P : nullptr;
    auto handoff = [&]() {
        ++hseq;
        vm_drain();
        __syncthreads();
        if (tid == 0 && !bad) {
            int verdict = 0;
            __hip_atomic_store(gflags + part, hseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // the budget is wall time (a part that is not resident at all never arrives;
            // one that is arrives within a column-iteration, tens of microseconds)
            const uint64_t t_wait = wall_clock64();
            for (int q = 0; q < A.P && !verdict; ++q) {
                if (q == part) continue;
                while (__hip_atomic_load(gflags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < hseq) {
                    if (wall_clock64() - t_wait >= (uint64_t)A.spinmax) {
                        verdict = 1;
                        __hip_atomic_store(A.abortf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            s_ch[4 * kRegMaxChunks] = verdict;
        }
        __syncthreads();
        bad = bad || s_ch[4 * kRegMaxChunks] != 0;
    };
    // SPLIT: chunk dots of the group, [hand-off parity][global chunk]
    const __amdgpu_buffer_rsrc_t xcs = __builtin_amdgcn_make_buffer_rsrc(
        SPLIT ? A.xch + (int64_t)group * 2 * kRegMaxChunks : A.pg, 0, 2 * kRegMaxChunks * 8, 0x00020000);

    // OpenBLAS finish of one dot (every wave computes it; lane = chunk)
    // lanes 4 t + l (t < T, l < 4) fold c4[l] of chunk t with all their LDS loads in
    // flight; lane 4 t collects its quad's four (DPP) and adds the chunk's FMA tail; the
    // chunks are summed in order from scalar reads (v_readlane), so the result is
    // wave-uniform without a broadcast
    auto finish = [&](const double *acc32all, const double *xa_all, const double *xb_all) -> double {
        const int tq = lane >> 2, l = lane & 3;
        const bool lv = tq < T;
        const int Lt = s_ch[kRegMaxChunks + (lv ? tq : 0)];
        const int n1 = Lt & ~15, n32t = n1 & ~31;
        const double *a32 = acc32all + tq * 32;  // dereferenced only when lv
        const double *xa = xa_all + tq * 32, *xb = xb_all + tq * 32;
        double cl = 0.0;
        if (lv && n1) {
            // b[4q + l] = acc[8q + l] + acc[8q + 4 + l] (+ the 16-block row 4q + l),
            // c4[l] = ((b[l] + b[4 + l]) + b[8 + l]) + b[12 + l]
            const bool blk = n1 > n32t;
            double av[4], bv[4], pa[4], pb[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                av[q] = a32[8 * q + l];
                bv[q] = a32[8 * q + 4 + l];
                pa[q] = blk ? xa[4 * q + l] : 0.0;
                pb[q] = blk ? xb[4 * q + l] : 0.0;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                double b = av[q] + bv[q];
                if (blk) b = __builtin_fma(pa[q], pb[q], b);
                cl = q == 0 ? b : cl + b;
            }
        }
        const double c0 = wide_quad_bcast<0>(cl), c1 = wide_quad_bcast<1>(cl);
        const double c2 = wide_quad_bcast<2>(cl), c3 = wide_quad_bcast<3>(cl);
        double dot = n1 ? (c0 + c2) + (c1 + c3) : 0.0;
        if (lv && l == 0) {
            const int nt = Lt - n1, ib = n1 - n32t;  // tail rows (< 16) after the 16-block
            for (int i0 = 0; i0 < nt; i0 += 4) {
                double ta[4], tb[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    ta[i] = i0 + i < nt ? xa[ib + i0 + i] : 0.0;
                    tb[i] = i0 + i < nt ? xb[ib + i0 + i] : 0.0;
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    if (i0 + i < nt) dot = __builtin_fma(tb[i], ta[i], dot);
            }
        }
        if constexpr (SPLIT) {
            // publish this part's chunk dots (wave 0, lane 4 t), hand off, then every wave
            // adds all Tg chunk dots of the column in global chunk order
            const int slot = ((hseq + 1) & 1) * kRegMaxChunks;
            if (tid < 64 && lv && l == 0)
                __builtin_amdgcn_raw_buffer_store_b64(
                    __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, dot), xcs,
                    (slot + t0g + tq) * 8, 0, 16);
            handoff();
            const double all = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(xcs, lane < Tg ? (slot + lane) * 8 : kOob, 0, 16));
            double total = 0.0;
            for (int tt = 0; tt < Tg; ++tt) total = total + wide_readlane(all, tt);
            return total;
        }
        if (T == 1) return wide_readlane(dot, 0);
        double total = 0.0;
        for (int tt = 0; tt < T; ++tt) total = total + wide_readlane(dot, 4 * tt);
        return total;
    };

    long long tp[5] = {0, 0, 0, 0, 0};
    long long tmark = wall_clock64();
    auto lap = [&](int ph) {
        const long long tn = wall_clock64();
        tp[ph] += tn - tmark;
        tmark = tn;
    };

    const int64_t ncols = (A.gate && *A.gate == 0) ? 0 : A.ncols;
    for (int64_t ci = group; ci < ncols; ci += ngroups) {
        const int64_t c = A.col0 + ci;
        double r[R], x[QR ? 1 : R], qr[QR && !QSX ? R : 1];
        // QR: x of the slots in this column's Xc rows (raw buffer; rows past n dropped)
        const __amdgpu_buffer_rsrc_t xrs =
            __builtin_amdgcn_make_buffer_rsrc(A.Xc + ci * A.ldn, 0, (int)(A.n * 8), 0x00020000);
        auto xload = [&](int u) -> double {
            return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xrs, base * 8, 256 * G * u, GS_CG_XAUX));
        };
        auto xstore = [&](int u, double v) {
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), xrs, base * 8, 256 * G * u,
                GS_CG_XAUX);
        };
        // QS: q of slot u to / from the Xc column (rows of slots past the lane's chain rows
        // are not this lane's: their offset lies past the buffer, so the store is dropped
        // and the load reads 0.0)
        auto qstore = [&](int u, double v) {
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), xrs,
                valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX);
        };
        auto qload = [&](int u) -> double {
            return __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(xrs, valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX));
        };
        // QSX: q scratch of this workgroup (the second half of A.pg, after every slot's p rows)
        const __amdgpu_buffer_rsrc_t qsr = __builtin_amdgcn_make_buffer_rsrc(
            A.pg + ((int64_t)gridDim.x + group) * A.ldn, 0, QSX ? (int)(A.n * 8) : 0, 0x00020000);
        auto q2store = [&](int u, double v) {
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), qsr,
                valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX);
        };
        auto q2load = [&](int u) -> double {
            return __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(qsr, valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX));
        };
        auto xload2 = [&](int u) -> double {
            return __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(xrs, valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX));
        };
        auto xstore2 = [&](int u, double v) {
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, v), xrs,
                valid(u) ? base * 8 : kOob, 256 * G * u, GS_CG_QAUX);
        };
        // r = b.copy(); rho_0 = b.b
        {
            launder();
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < R; ++u) {
                if constexpr (!QR) x[u] = 0.0;
                else qr[u] = 0.0;
                r[u] = valid(u) ? A.Rr[(int64_t)rowof(u) * A.ld + c] : 0.0;
                chain_step(acc, r[u], r[u], u, true);
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
            if constexpr (SPLIT) poff = (it & 1) * (int)A.ldn * 8;
            lap(4);
            // p = beta p + r (two roundings); x += alpha_{it-1} p_{it-1} rides along
            launder();
            // slots u < ulds: p at lds0 + 256 G u (their stores need no valid test either:
            // a lane's LDS-prefix rows are its own chain rows or its chunk's)
            // (tried, round 3: the global p rows' loads without the VMEM drain, or
            // branch-free with a select -- 43.85 / 43.70 vs 43.81 us per column-iteration,
            // profiles/r03e/: the drain is not what the p pass waits on)
            auto pload = [&](int u) -> double {
                return u < ulds ? lds_at(lds0() + 256u * G * u) : valid(u) ? ldc(code_of(rowof(u))) : 0.0;
            };
            auto pstore = [&](int u, double v) {
                if (u < ulds) lds_put(lds0() + 256u * G * u, v);
                else stc(code_of(rowof(u)), v);
                if constexpr (SPLIT) {
                    if (valid(u)) publish(rowof(u), v);
                }
            };
            if (it == 0) {
#pragma unroll
                for (int u = 0; u < R; ++u)
                    if (valid(u)) pstore(u, r[u]);
            } else {
                double pb4[R];  // p_old, kPreP slots ahead (each slot reads and writes only its row)
#pragma unroll
                for (int u = 0; u < kPreP && u < R; ++u) pb4[u] = pload(u);
                if constexpr (!SPLIT) {
                    // two straight-line passes: every slot reads p_old from LDS (slots past
                    // the wave's LDS prefix read the zero slot and store to the scratch
                    // slot: x += alpha * 0 and p to scratch change nothing), then the slots
                    // past the prefix redo their update from the global p rows.  No branch
                    // between a prefetch and its use, so the waits count only what is needed.
                    const uint32_t zaddr = (uint32_t)zslot * 8u, saddr = (uint32_t)(zslot + 1) * 8u;  // the scratch slot
                    double pf[R];
#pragma unroll
                    for (int u = 0; u < kPreP && u < R; ++u) pf[u] = lds_at(u < ulds ? lds0() + 256u * G * u : zaddr);
#pragma unroll
                    for (int u = 0; u < R; ++u) {
                        if (u + kPreP < R)
                            pf[u + kPreP] = lds_at(u + kPreP < ulds ? lds0() + 256u * G * (u + kPreP) : zaddr);
                        const double po = pf[u];
                        if constexpr (!QR) {
                            const double t1 = alpha_prev * po;
                            x[u] = x[u] + t1;
                            asm volatile("" : "+v"(x[u]));  // now, not deferred to the second pass
                        }
                        const double pb = po * beta;
                        lds_put(u < ulds && valid(u) ? lds0() + 256u * G * u : saddr, pb + r[u]);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    launder();
                    if constexpr (V2 && GS_PGRP > 0) {
                        // the slots past the prefix in groups of GS_PGRP: all their p_old loads (LDS
                        // or the global rows) issued, one wait, then the updates -- one memory
                        // round trip per group instead of one per slot
                        constexpr int kGrp = GS_PGRP;
#pragma unroll
                        for (int u0 = 0; u0 < R; u0 += kGrp) {
                            if (u0 + kGrp <= ulds) continue;  // wave-uniform: the group is in the prefix
                            double pog[kGrp > 0 ? kGrp : 1];
#pragma unroll
                            for (int k = 0; k < kGrp; ++k) {
                                const int u = u0 + k;
                                if (u >= R) break;
                                const int cd = code_of(rowof(u));
                                const bool gl = cd >= 0x8000 && u >= ulds && valid(u);
                                const double lv = spl[cd < 0x8000 ? cd : zslot];
                                const double gv = __builtin_bit_cast(
                                    double, __builtin_amdgcn_raw_buffer_load_b64(
                                                prs, gl ? (cd & 0x7fff) * 8 + poff : kOob, 0, kAux));
                                pog[k] = cd < 0x8000 ? lv : gv;
                            }
                            vm_drain();
#pragma unroll
                            for (int k = 0; k < kGrp; ++k) {
                                const int u = u0 + k;
                                if (u >= R) break;
                                if (u >= ulds && valid(u)) {
                                    const double po = pog[k];
                                    if constexpr (!QR) {
                                        const double t1 = alpha_prev * po;
                                        x[u] = x[u] + t1;
                                    }
                                    const double pb = po * beta;
                                    pstore(u, pb + r[u]);
                                }
                            }
                        }
                    } else {
#pragma unroll
                    for (int u = 0; u < R; ++u) {
                        if (u >= ulds && valid(u)) {
                            const double po = ldc(code_of(rowof(u)));
                            if constexpr (!QR) {
                                const double t1 = alpha_prev * po;
                                x[u] = x[u] + t1;
                            }
                            const double pb = po * beta;
                            pstore(u, pb + r[u]);
                        }
                    }
                    }
                } else
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPreP < R) pb4[u + kPreP] = pload(u + kPreP);
                    if (valid(u)) {
                        const double po = pb4[u];
                        if constexpr (!QR) {
                            const double t1 = alpha_prev * po;
                            x[u] = x[u] + t1;
                        }
                        const double pb = po * beta;
                        pstore(u, pb + r[u]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (tail) {
                if (it == 0) {
                    stc(code_of(trow), side_r[tix]);
                    publish(trow, side_r[tix]);
                } else {
                    const double po = ldc(code_of(trow));
                    if constexpr (!QR) {
                        const double t1 = alpha_prev * po;
                        side_x[tix] = side_x[tix] + t1;
                    }
                    const double pb = po * beta;
                    stc(code_of(trow), pb + side_r[tix]);
                    publish(trow, pb + side_r[tix]);
                }
            }
            if constexpr (SPLIT) {
                handoff();  // every part's p published before any SpMV reads it
            } else {
                __syncthreads();
            }
            lap(0);
            // q = L_reg p and the chains of p.q
            {
                launder();
                double acc = 0.0;
                uint4 eb[R];  // ELL rows and lengths (V2: diagonals), kPre slots ahead
                int lb[R];
                double db[R];
#pragma unroll
                for (int u = 0; u < kPre && u < R; ++u) {
                    eb[u] = ell_row(u);
                    if constexpr (V2) db[u] = diag_row(u);
                    else lb[u] = len_row(u);
                }
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPre < R) {
                        eb[u + kPre] = ell_row(u + kPre);
                        if constexpr (V2) db[u + kPre] = diag_row(u + kPre);
                        else lb[u + kPre] = len_row(u + kPre);
                    }
                    double pv = 0.0, qv = 0.0;
                    if constexpr (V2) {
                        if (valid(u)) qv = spmv2(rowof(u), eb[u], db[u], pv, u);
                    } else if (valid(u)) qv = spmv(rowof(u), eb[u], lb[u], pv, u);
                    if constexpr (QSX) q2store(u, qv);
                    else if constexpr (QR) qr[u] = qv;
                    if constexpr (QS) qstore(u, qv);
                    chain_step(acc, pv, qv, u);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_pq[chain] = acc;
                if (tail) {
                    double pt;
                    side_q[tix] = spmv(trow, A.ell[trow], (int)A.rlen[trow], pt, -1);
                    side_p[tix] = pt;
                }
            }
            __syncthreads();
            lap(1);
            const double pq = finish(acc_pq, side_p, side_q);
            const double alpha = rho_cur / pq;
            lap(2);
            // QSX: x += alpha p, r -= alpha q with q, x and the global p rows read kPq slots
            // ahead (the LDS p rows read in place), chains of r.r
            if constexpr (QSX) {
                launder();
                double acc = 0.0;
                constexpr int kPq = GS_CG_QPRE;
                double qb[R], xb[R], pgb[R];
                auto pre = [&](int u) {
                    qb[u] = q2load(u);
                    xb[u] = it > 0 ? xload2(u) : 0.0;
                    // global p rows: their buffer load now (LDS rows read 0 here, in place below)
                    const int cd = u < ulds ? 0 : code_of(rowof(u));
                    pgb[u] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                                                            prs, cd >= 0x8000 && valid(u) ? (cd & 0x7fff) * 8 + poff : kOob,
                                                            0, kAux));
                };
#pragma unroll
                for (int u = 0; u < kPq && u < R; ++u) pre(u);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPq < R) pre(u + kPq);
                    if (valid(u)) {
                        double pu;
                        if (u < ulds) {
                            pu = lds_at(lds0() + 256u * G * u);
                        } else {
                            const int cd = code_of(rowof(u));
                            const double lv = spl[cd < 0x8000 ? cd : zslot];
                            pu = cd < 0x8000 ? lv : pgb[u];
                        }
                        const double t1 = alpha * pu;
                        xstore2(u, xb[u] + t1);
                        const double t2 = alpha * qb[u];
                        r[u] = r[u] - t2;
                    }
                    chain_step(acc, r[u], r[u], u, true);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_rr[chain] = acc;
                if (tail) {
                    const double t1 = alpha * side_p[tix];
                    side_x[tix] = side_x[tix] + t1;
                    const double t2 = alpha * side_q[tix];
                    side_r[tix] = side_r[tix] - t2;
                }
            } else
            // QR: x += alpha p (x from / to Xc, p from LDS), r -= alpha q (q in registers),
            // chains of r.r
            if constexpr (QR) {
                launder();
                double acc = 0.0;
                double xb[R];  // x, kPre slots ahead (no read in the first iteration: x == 0)
                if (it > 0) {
#pragma unroll
                    for (int u = 0; u < kPre && u < R; ++u) xb[u] = xload(u);
                }
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (it > 0 && u + kPre < R) xb[u + kPre] = xload(u + kPre);
                    if (valid(u)) {
                        const double t1 = alpha * pload(u);
                        xstore(u, (it > 0 ? xb[u] : 0.0) + t1);
                        const double t2 = alpha * qr[u];
                        r[u] = r[u] - t2;
                    }
                    chain_step(acc, r[u], r[u], u, true);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_rr[chain] = acc;
                if (tail) {
                    const double t1 = alpha * side_p[tix];
                    side_x[tix] = side_x[tix] + t1;
                    const double t2 = alpha * side_q[tix];
                    side_r[tix] = side_r[tix] - t2;
                }
            } else if constexpr (QS) {
                // r -= alpha q (q from the SpMV pass, read back from the Xc column), chains of r.r
                launder();
                double acc = 0.0;
                constexpr int kPq = GS_CG_QPRE;
                double qb[R];
#pragma unroll
                for (int u = 0; u < kPq && u < R; ++u) qb[u] = qload(u);
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPq < R) qb[u + kPq] = qload(u + kPq);
                    if (valid(u)) {
                        const double t2 = alpha * qb[u];
                        r[u] = r[u] - t2;
                    }
                    chain_step(acc, r[u], r[u], u, true);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_rr[chain] = acc;
                if (tail) {
                    const double t2 = alpha * side_q[tix];
                    side_r[tix] = side_r[tix] - t2;
                }
            } else
            // r -= alpha q (q recomputed), chains of r.r
            {
                launder();
                double acc = 0.0;
                uint4 eb[R];
                int lb[R];
                double db[R];
#pragma unroll
                for (int u = 0; u < kPre && u < R; ++u) {
                    eb[u] = ell_row(u);
                    if constexpr (V2) db[u] = diag_row(u);
                    else lb[u] = len_row(u);
                }
#pragma unroll
                for (int u = 0; u < R; ++u) {
                    if (u + kPre < R) {
                        eb[u + kPre] = ell_row(u + kPre);
                        if constexpr (V2) db[u + kPre] = diag_row(u + kPre);
                        else lb[u + kPre] = len_row(u + kPre);
                    }
                    if (valid(u)) {
                        double pu;
                        const double q = V2 ? spmv2(rowof(u), eb[u], db[u], pu, u)
                                            : spmv(rowof(u), eb[u], lb[u], pu, u);
                        const double t2 = alpha * q;
                        r[u] = r[u] - t2;
                    }
                    chain_step(acc, r[u], r[u], u, true);
                    __builtin_amdgcn_sched_barrier(0);
                }
                if (g == 0 && live) acc_rr[chain] = acc;
                if (tail) {
                    double pt;
                    const double t2 = alpha * spmv(trow, A.ell[trow], (int)A.rlen[trow], pt, -1);
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
        if constexpr (QR) {  // x is in place after any iteration
            if (bn == 0.0 || done == 0) {
#pragma unroll
                for (int u = 0; u < R; ++u)
                    if (valid(u)) xstore(u, bn == 0.0 ? r[u] : 0.0);
            }
            if (tail) xo[trow] = bn == 0.0 ? side_r[tix] : done == 0 ? 0.0 : side_x[tix];
        } else {
#pragma unroll
        for (int u = 0; u < R; ++u)
            if (valid(u)) {
                const int row = rowof(u);
                double v;
                if (bn == 0.0) v = r[u];
                else if (done == 0) v = 0.0;
                else {
                    const double t1 = alpha_prev * ldc(code_of(row));
                    v = (done > 1 ? x[u] : 0.0) + t1;
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
        }
        if (tid == 0 && part == 0) A.iters[c] = done;
        __syncthreads();  // the next column's b.b chains reuse acc_rr / side_r
    }
    if (A.prof && blockIdx.x == 0 && tid == 0)
        for (int i = 0; i < 5; ++i) A.prof[i] = tp[i];
}

// one launch: R row slots (16 / 24 / 32 / 44), unit or weighted form
#define GS_REGWIDE_LAUNCH_DEF(G_)                                                             \
    void regwide_launch_g##G_(const RegArgs &A, int R, bool unit, size_t dyn, unsigned slots, \
                              hipStream_t s) {                                                \
        auto go = [&](auto kern) {                                                            \
            GS_HIP(hipFuncSetAttribute((const void *)kern,                                    \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn)); \
            kern<<<slots, kRegThreads, dyn, s>>>(A);                                          \
        };                                                                                    \
        auto pick = [&](auto qr) {                                                            \
            constexpr bool Q = decltype(qr)::value;                                           \
            if (unit) {                                                                       \
                if (R == 16) go(k_cg_regwide<G_, 16, true, Q>);                               \
                else if (R == 24) go(k_cg_regwide<G_, 24, true, Q>);                          \
                else if (R == 32) go(k_cg_regwide<G_, 32, true, Q>);                          \
                else go(k_cg_regwide<G_, 44, true, Q>);                                       \
            } else {                                                                          \
                if (R == 16) go(k_cg_regwide<G_, 16, false, Q>);                              \
                else if (R == 24) go(k_cg_regwide<G_, 24, false, Q>);                         \
                else if (R == 32) go(k_cg_regwide<G_, 32, false, Q>);                         \
                else go(k_cg_regwide<G_, 44, false, Q>);                                      \
            }                                                                                 \
        };                                                                                    \
        (void)A.qreg; /* whole columns keep x in registers (the q-in-registers form of */     \
        /* round 2 lives on only in the split tail; GS_CG_XG: x in Xc, q stored) */           \
        pick(std::integral_constant<bool, (bool)GS_CG_XG>{});                                 \
    }

// one launch of the split form (q in registers), grid = groups x A.P workgroups
#define GS_REGWIDE_SPLIT_DEF(G_)                                                               \
    void regwide_split_launch_g##G_(const RegArgs &A, int R, bool unit, size_t dyn,            \
                                    unsigned grid, hipStream_t s) {                            \
        auto go = [&](auto kern) {                                                             \
            GS_HIP(hipFuncSetAttribute((const void *)kern,                                     \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn));  \
            kern<<<grid, kRegThreads, dyn, s>>>(A);                                            \
        };                                                                                     \
        if (unit) {                                                                            \
            if (R == 16) go(k_cg_regwide<G_, 16, true, true, true>);                           \
            else if (R == 24) go(k_cg_regwide<G_, 24, true, true, true>);                      \
            else if (R == 32) go(k_cg_regwide<G_, 32, true, true, true>);                      \
            else go(k_cg_regwide<G_, 44, true, true, true>);                                   \
        } else {                                                                               \
            if (R == 16) go(k_cg_regwide<G_, 16, false, true, true>);                          \
            else if (R == 24) go(k_cg_regwide<G_, 24, false, true, true>);                     \
            else if (R == 32) go(k_cg_regwide<G_, 32, false, true, true>);                     \
            else go(k_cg_regwide<G_, 44, false, true, true>);                                  \
        }                                                                                      \
    }

}  // namespace gs
