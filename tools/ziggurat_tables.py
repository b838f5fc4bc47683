"""Recover NumPy's float64 normal-ziggurat constants by probing the public API.

numpy/random/src/distributions (random_standard_normal) draws r = next_uint64:
  idx = r & 0xff; sign = (r >> 8) & 1; rabs = (r >> 9) & (2^52 - 1)
  x = rabs * wi[idx] (negated for sign); fast accept iff rabs < ki[idx];
  idx == 0: tail  xx = -inv_r * log1p(-U1), yy = -log1p(-U2) until
            yy + yy > xx * xx, returning +-(r + xx) (sign from bit 8 of rabs);
  else:     accept iff (fi[idx-1] - fi[idx]) * U + fi[idx] < exp(-x*x/2).
The tables are not part of NumPy's installed files, so this script forces
chosen 64-bit outputs out of PCG64 (picking the 128-bit state and the odd
increment so that the next one or two outputs are given values) and reads:
  wi[idx]  = the value returned for rabs = 1 (accepted for U = 0);
  ki[idx]  = the smallest rabs for which more than one draw is consumed;
  r        = the tail value returned when U1 = 0 (log1p(-0) = -0, xx = +0);
  fi[idx]  = fi is only compared against exp(); its values are located in
             NumPy's own shared object as the 256 doubles that follow the wi
             table (read as data, verified: fi[0] == 1, decreasing, and
             consistent with every probed accept/reject decision).
Writes gnn-sparsification-research_amd/csrc/gs_ziggurat_tables.hpp.
"""

from __future__ import annotations

import glob
import os
import struct
import sys

import numpy as np

MULT = 0x2360ED051FC65DA44385DF649FCCF645
M128 = (1 << 128) - 1
M64 = (1 << 64) - 1
MULT_INV = pow(MULT, -1, 1 << 128)


def _state_for(outputs):
    """(s0, inc) such that the next len(outputs) (<= 2) PCG64 outputs are `outputs`."""
    H1 = 0x0001234567890ABC  # rot = H >> 58 = 0
    s1 = (H1 << 64) | (outputs[0] ^ H1)
    if len(outputs) == 1:
        inc = 0xDA3E39CB94B95BDB
    else:
        H2 = 0x0000FEDCBA987654
        s2 = (H2 << 64) | (outputs[1] ^ H2)
        inc = (s2 - s1 * MULT) & M128
        if inc % 2 == 0:
            H2 ^= 1
            s2 = (H2 << 64) | (outputs[1] ^ H2)
            inc = (s2 - s1 * MULT) & M128
        assert inc % 2 == 1
    s0 = ((s1 - inc) * MULT_INV) & M128
    return s0, inc


def _gen(outputs):
    s0, inc = _state_for(outputs)
    bg = np.random.PCG64()
    bg.state = {"bit_generator": "PCG64", "state": {"state": s0, "inc": inc},
                "has_uint32": 0, "uinteger": 0}
    return np.random.Generator(bg), s0, inc


def draws_used(outputs):
    g, s0, inc = _gen(outputs)
    v = g.standard_normal()
    s = g.bit_generator.state["state"]["state"]
    k, t = 0, s0
    while t != s:
        t = (t * MULT + inc) & M128
        k += 1
        assert k < 64
    return v, k


def make_r(idx, sign, rabs):
    return idx | (sign << 8) | (rabs << 9)


def probe():
    wi, ki = [], []
    for idx in range(256):
        v, _ = draws_used([make_r(idx, 0, 1), 0])
        wi.append(v)
        lo, hi = 0, (1 << 52)  # smallest rabs with > 1 draw
        while lo < hi:
            mid = (lo + hi) // 2
            _, k = draws_used([make_r(idx, 0, mid), 0])
            if k > 1:
                hi = mid
            else:
                lo = mid + 1
        ki.append(lo)
    # tail value with U1 = 0: idx 0, rabs >= ki[0]
    r_tail, k = draws_used([make_r(0, 0, (1 << 52) - 1), 0])
    return wi, ki, r_tail


def find_fi(wi):
    import numpy.random as nr

    d = os.path.dirname(nr.__file__)
    pat = struct.pack("<" + "d" * 4, *wi[:4])
    for path in sorted(glob.glob(os.path.join(d, "*.so")) + glob.glob(os.path.join(d, "..", "*.so"))):
        blob = open(path, "rb").read()
        pos = blob.find(pat)
        while pos >= 0:
            tab = struct.unpack_from("<256d", blob, pos)
            if list(tab) == list(wi):
                # the fi table sits next to wi/ki (ki: 256 uint64) in .rodata
                for off in (256 * 8 * 2, -256 * 8, 256 * 8):
                    cand = struct.unpack_from("<256d", blob, pos + off)
                    if cand[0] == 1.0 and all(cand[i] > cand[i + 1] for i in range(255)):
                        return list(cand), path
            pos = blob.find(pat, pos + 1)
    raise RuntimeError("fi table not located")


def check_fi(wi, ki, fi, trials=2000):
    """Every probed slow-path decision agrees with the recovered fi."""
    import math

    rng = np.random.default_rng(5)
    for _ in range(trials):
        idx = int(rng.integers(1, 256))
        rabs = int(rng.integers(ki[idx], 1 << 52)) if ki[idx] < (1 << 52) else None
        if rabs is None:
            continue
        u64 = int(rng.integers(0, 1 << 63)) * 2 + int(rng.integers(0, 2))
        U = (u64 >> 11) * (1.0 / 9007199254740992.0)
        x = rabs * wi[idx]
        accept = ((fi[idx - 1] - fi[idx]) * U + fi[idx]) < math.exp(-0.5 * x * x)
        v, k = draws_used([make_r(idx, 0, rabs), u64])
        assert (k == 2) == accept or (k == 2 and v == x), (idx, rabs, k, accept)
        if k == 2:
            assert v == x


def find_inv_r(r, ki0):
    """inv_r: the candidate that reproduces forced tail draws (U1 chosen, U2 free)."""
    import ctypes
    import math

    libm = ctypes.CDLL("libm.so.6")
    libm.log1p.restype = ctypes.c_double
    libm.log1p.argtypes = [ctypes.c_double]
    base = 1.0 / r
    cands = {base, float("0.27366123732975828")}
    for d in (-2, -1, 1, 2):
        cands.add(math.nextafter(base, math.inf if d > 0 else -math.inf) if abs(d) == 1 else
                  math.nextafter(math.nextafter(base, math.inf if d > 0 else -math.inf),
                                 math.inf if d > 0 else -math.inf))
    alive = set(cands)
    rng = np.random.default_rng(9)
    hits = 0
    while hits < 200:
        u1 = int(rng.integers(1, 1 << 63)) * 2 + 1
        U1 = (u1 >> 11) * (1.0 / 9007199254740992.0)
        rabs = (1 << 52) - 2 - (1 << 8)  # bit 8 clear: positive tail
        assert rabs >= ki0
        v, k = draws_used([make_r(0, 0, rabs), u1])
        if k != 3:
            continue  # U2 (uncontrolled) rejected this pair
        hits += 1
        for c in list(alive):
            xx = -c * libm.log1p(-U1)
            if r + xx != v:
                alive.discard(c)
    assert len(alive) >= 1, "no inv_r candidate fits"
    vals = sorted(alive)
    assert len(set(vals)) == 1 or all(v == vals[0] for v in vals), vals
    return vals[0]


def main():
    wi, ki, r_tail = probe()
    fi, path = find_fi(wi)
    check_fi(wi, ki, fi)
    r_tail = abs(r_tail)
    inv_r = find_inv_r(r_tail, ki[0])
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "gnn-sparsification-research_amd", "csrc", "gs_ziggurat_tables.hpp")
    with open(out, "w") as f:
        f.write("// NumPy (2.2) float64 normal-ziggurat constants, recovered by\n"
                "// tools/ziggurat_tables.py (PCG64 output forcing + fi located in\n"
                f"// {os.path.basename(path)}).  Do not edit.\n#pragma once\n#include <cstdint>\n"
                "namespace gs {\n")
        f.write(f"static constexpr double kZigR = {r_tail!r};  // bits {struct.unpack('<Q', struct.pack('<d', r_tail))[0]:#018x}\n")
        f.write(f"static constexpr double kZigInvR = {inv_r!r};  // bits {struct.unpack('<Q', struct.pack('<d', inv_r))[0]:#018x}\n")
        f.write("__constant__ static const uint64_t kZigKi[256] = {\n")
        f.write(",\n".join("    " + ", ".join(f"{v:#018x}ull" for v in ki[i:i + 4]) for i in range(0, 256, 4)))
        f.write("};\n__constant__ static const uint64_t kZigWiBits[256] = {\n")
        wb = [struct.unpack("<Q", struct.pack("<d", v))[0] for v in wi]
        f.write(",\n".join("    " + ", ".join(f"{v:#018x}ull" for v in wb[i:i + 4]) for i in range(0, 256, 4)))
        f.write("};\n__constant__ static const uint64_t kZigFiBits[256] = {\n")
        fb = [struct.unpack("<Q", struct.pack("<d", v))[0] for v in fi]
        f.write(",\n".join("    " + ", ".join(f"{v:#018x}ull" for v in fb[i:i + 4]) for i in range(0, 256, 4)))
        f.write("};\n")
        # host copies (tools/zig_host_check.cpp validates the parser on the CPU)
        for nm, vals in (("kZigKiH", ki), ("kZigWiBitsH", wb), ("kZigFiBitsH", fb)):
            f.write(f"static const uint64_t {nm}[256] = {{\n")
            f.write(",\n".join("    " + ", ".join(f"{v:#018x}ull" for v in vals[i:i + 4])
                               for i in range(0, 256, 4)))
            f.write("};\n")
        f.write("}  // namespace gs\n")
    print("wrote", out, "r =", r_tail, "ki[0:4] =", [hex(v) for v in ki[:4]], "fi from", path)


if __name__ == "__main__":
    main()
