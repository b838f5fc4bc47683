// gs_pairwise.hpp -- NumPy's pairwise summation on the device.
//
// numpy/_core/src/umath/loops_utils.h.src pairwise_sum_@TYPE@, as reached by
// np.sum(..., axis=1) / np.linalg.norm(..., axis=1) on contiguous rows
// (metrics.py:293, :344, :351), with the reduce's identity 0 added in front:
//   n < 8      : r = 0; r += a[i] sequentially
//   n <= 128   : 8 strided accumulators r[j] = a[j] + a[j+8] + ...,
//                res = ((r0+r1)+(r2+r3)) + ((r4+r5)+(r6+r7)), then the tail
//   otherwise  : n2 = n/2 - (n/2)%8; pw(a[:n2]) + pw(a[n2:])
// get(i) must return the already-rounded i-th term (the caller forms
// products / squared differences with separate roundings, -ffp-contract=off).
#pragma once
#include <hip/hip_runtime.h>

namespace gs {

template <class T, class F>
__device__ __forceinline__ T pw_leaf(int64_t off, int64_t n, F &get) {
    if (n < 8) {
        T r = T(0);
        for (int64_t i = 0; i < n; ++i) r = r + get(off + i);
        return r;
    }
    T r0 = get(off + 0), r1 = get(off + 1), r2 = get(off + 2), r3 = get(off + 3);
    T r4 = get(off + 4), r5 = get(off + 5), r6 = get(off + 6), r7 = get(off + 7);
    int64_t i = 8, lim = n - (n % 8);
    for (; i < lim; i += 8) {
        r0 = r0 + get(off + i + 0);
        r1 = r1 + get(off + i + 1);
        r2 = r2 + get(off + i + 2);
        r3 = r3 + get(off + i + 3);
        r4 = r4 + get(off + i + 4);
        r5 = r5 + get(off + i + 5);
        r6 = r6 + get(off + i + 6);
        r7 = r7 + get(off + i + 7);
    }
    T res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; ++i) res = res + get(off + i);
    return res;
}

// Iterative post-order walk of the pairwise tree (depth <= 48 for n < 2^55).
template <class T, class F>
__device__ T pw_sum(int64_t n, F get) {
    if (n <= 128) return pw_leaf<T>(0, n, get);
    int64_t off_s[48], n_s[48];
    T left_s[48];
    unsigned char st_s[48];
    int sp = 0;
    off_s[0] = 0;
    n_s[0] = n;
    st_s[0] = 0;
    T ret = T(0);
    for (;;) {
        int64_t off = off_s[sp], nn = n_s[sp];
        int64_t n2 = nn / 2;
        n2 -= n2 % 8;
        if (st_s[sp] == 0) {
            if (nn <= 128) {
                ret = pw_leaf<T>(off, nn, get);
            } else {
                st_s[sp] = 1;
                ++sp;
                off_s[sp] = off;
                n_s[sp] = n2;
                st_s[sp] = 0;
                continue;
            }
        } else if (st_s[sp] == 1) {
            left_s[sp] = ret;
            st_s[sp] = 2;
            ++sp;
            off_s[sp] = off + n2;
            n_s[sp] = nn - n2;
            st_s[sp] = 0;
            continue;
        } else {
            ret = left_s[sp] + ret;
        }
        if (sp == 0) return ret;
        --sp;
    }
}

}  // namespace gs
