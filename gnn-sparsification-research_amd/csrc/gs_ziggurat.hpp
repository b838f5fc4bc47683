// gs_ziggurat.hpp -- NumPy's Generator(PCG64).standard_normal stream, bit for bit.
//
// metrics.py:232,272 draws R = default_rng(seed).standard_normal((m, k)).
// NumPy 2.2: PCG64 (128-bit LCG, multiplier 0x2360ED051FC65DA44385DF649FCCF645,
// XSL-RR output, state advanced before each output) feeding
// random_standard_normal's 256-level ziggurat (tables: gs_ziggurat_tables.hpp,
// recovered by tools/ziggurat_tables.py).  One "attempt" consumes:
//   1 draw  : fast accept (rabs < ki[idx])                        -> value
//   2 draws : idx > 0 wedge test with U = next_double             -> value | retry
//   1 + 2j  : idx == 0 tail, j pairs (U1, U2) until yy+yy > xx*xx  -> value
// The tail uses glibc's log1p (NumPy's npy_log1p is libm's): restated below
// with glibc 2.35's exact operation order (fdlibm algorithm, Estrin-split
// polynomial), bit-identical on 10^6 inputs in (-1, 0].  exp() only decides
// the wedge test, where a last-ulp difference flips a decision with
// probability ~2^-52 per test.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "gs_ziggurat_tables.hpp"

namespace gs {

typedef unsigned __int128 u128;

static constexpr uint64_t kPcgMulHi = 0x2360ED051FC65DA4ull;
static constexpr uint64_t kPcgMulLo = 0x4385DF649FCCF645ull;

__host__ __device__ __forceinline__ u128 pcg_mult() { return ((u128)kPcgMulHi << 64) | kPcgMulLo; }

__host__ __device__ __forceinline__ uint64_t pcg_output(u128 s) {
    uint64_t hi = (uint64_t)(s >> 64), lo = (uint64_t)s;
    unsigned rot = (unsigned)(s >> 122);
    uint64_t v = hi ^ lo;
    return (v >> rot) | (v << ((64u - rot) & 63u));
}

struct Pcg64 {
    u128 s, inc;
    __host__ __device__ __forceinline__ uint64_t next() {
        s = s * pcg_mult() + inc;
        return pcg_output(s);
    }
    __host__ __device__ __forceinline__ double next_double() {
        return (double)(next() >> 11) * (1.0 / 9007199254740992.0);
    }
};

// state after `delta` steps (pcg_advance_lcg_128)
__host__ __device__ inline u128 pcg_advance(u128 s, u128 inc, uint64_t delta) {
    u128 acc_mult = 1, acc_plus = 0, cur_mult = pcg_mult(), cur_plus = inc;
    while (delta > 0) {
        if (delta & 1) {
            acc_mult *= cur_mult;
            acc_plus = acc_plus * cur_mult + cur_plus;
        }
        cur_plus = (cur_mult + 1) * cur_plus;
        cur_mult *= cur_mult;
        delta >>= 1;
    }
    return acc_mult * s + acc_plus;
}

__host__ __device__ __forceinline__ int32_t hi_word(double x) {
    return (int32_t)((uint64_t)__builtin_bit_cast(uint64_t, x) >> 32);
}
__host__ __device__ __forceinline__ double set_hi_word(double x, int32_t h) {
    uint64_t b = __builtin_bit_cast(uint64_t, x);
    b = ((uint64_t)(uint32_t)h << 32) | (b & 0xffffffffull);
    return __builtin_bit_cast(double, b);
}

// glibc 2.35 sysdeps/ieee754/dbl-64/s_log1p.c as compiled for x86-64 (order
// of every operation matches its object code; needs -ffp-contract=off).
__host__ __device__ inline double glibc_log1p(double x) {
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                 Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                 Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                 Lp7 = 1.479819860511658591e-01;
    double hfsq, f = 0, c = 0, s, z, R, u;
    int32_t k, hx, hu = 0, ax;
    hx = hi_word(x);
    ax = hx & 0x7fffffff;
    k = 1;
    if (hx < 0x3FDA827A) {
        if (ax >= 0x3ff00000) {
            if (x == -1.0) return -__builtin_inf();
            return __builtin_nan("");
        }
        if (ax < 0x3e200000) {
            if (ax < 0x3c900000) return x;
            return x - (x * x) * 0.5;
        }
        if (hx > 0 || hx <= (int32_t)0xbfd2bec4) {
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (hx >= 0x7ff00000) return x + x;
    if (k != 0) {
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = hi_word(u);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);
            c /= u;
        } else {
            u = x;
            hu = hi_word(u);
            k = (hu >> 20) - 1023;
            c = 0;
        }
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = set_hi_word(u, hu | 0x3ff00000);
        } else {
            k += 1;
            u = set_hi_word(u, hu | 0x3fe00000);
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    hfsq = (0.5 * f) * f;
    if (hu == 0) {
        if (f == 0.0) {
            if (k == 0) return 0.0;
            return ((double)k * ln2_lo + c) + (double)k * ln2_hi;
        }
        R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return (double)k * ln2_hi - ((R - ((double)k * ln2_lo + c)) - f);
    }
    s = f / (2.0 + f);
    z = s * s;
    double z2 = z * z, z4 = z2 * z2, z6 = z4 * z2;
    double t1 = (Lp3 * z + Lp2) * z2;
    t1 = t1 + Lp1 * z;
    double t2 = (Lp5 * z + Lp4) * z4;
    double t3 = (Lp7 * z + Lp6) * z6;
    R = (t1 + t2) + t3;
    double w = s * (hfsq + R);
    if (k == 0) return f - (hfsq - w);
    return (double)k * ln2_hi - ((hfsq - (((double)k * ln2_lo + c) + w)) - f);
}

template <bool DEV>
__host__ __device__ __forceinline__ uint64_t zig_ki(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return kZigKi[i];
#else
    return kZigKiH[i];
#endif
}
template <bool DEV>
__host__ __device__ __forceinline__ double zig_wi(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_bit_cast(double, kZigWiBits[i]);
#else
    return __builtin_bit_cast(double, kZigWiBitsH[i]);
#endif
}
template <bool DEV>
__host__ __device__ __forceinline__ double zig_fi(int i) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_bit_cast(double, kZigFiBits[i]);
#else
    return __builtin_bit_cast(double, kZigFiBitsH[i]);
#endif
}

// One ziggurat attempt from the current stream position.  Returns the number
// of draws consumed; *produced says whether a normal was returned (*val).
template <bool DEV = true>
__host__ __device__ inline int zig_attempt(Pcg64 &g, bool *produced, double *val) {
    uint64_t r = g.next();
    int idx = (int)(r & 0xff);
    r >>= 8;
    int sign = (int)(r & 0x1);
    uint64_t rabs = (r >> 1) & 0x000fffffffffffffull;
    double x = (double)rabs * zig_wi<DEV>(idx);
    if (sign & 0x1) x = -x;
    if (rabs < zig_ki<DEV>(idx)) {
        *produced = true;
        *val = x;
        return 1;
    }
    if (idx == 0) {
        int used = 1;
        for (;;) {
            double xx = -kZigInvR * glibc_log1p(-g.next_double());
            double yy = -glibc_log1p(-g.next_double());
            used += 2;
            if (yy + yy > xx * xx) {
                *produced = true;
                *val = ((rabs >> 8) & 0x1) ? -(kZigR + xx) : kZigR + xx;
                return used;
            }
            if (used > 1 << 20) {  // unreachable in practice; keeps the loop bounded
                *produced = false;
                return used;
            }
        }
    }
    double lhs = (zig_fi<DEV>(idx - 1) - zig_fi<DEV>(idx)) * g.next_double() + zig_fi<DEV>(idx);
    double rhs = ::exp(-0.5 * x * x);
    *produced = lhs < rhs;
    *val = x;
    return 2;
}

}  // namespace gs
