"""CPU model of the LDS bank conflicts of k_cg_regwide's SpMV gathers (V2 unit form,
512 threads, G = 2) on a graph, for the current p layout and candidate swizzles.

ds_read_b64 serves a wave in two 32-lane groups; the bank of double slot x is
x mod 32 (MI355X_MICROARCH.md LDS table); each extra distinct address on a bank
within a group costs one LDS cycle.  Counts the cycles of the 8 entry gathers of
every slot of every chunk (one column-iteration's SpMV pass), conflict-free = 2 per
wave-instruction.

usage: lds_bank_sim.py [T]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "gnn-sparsification-research_amd"))
from gsparse import graphs  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 8
NT, G, KMAX = 512, 2, 16
ei = graphs.roman_like()
n = 22_662
keys = np.unique(ei[0] * n + ei[1])
rows, cols = keys // n, keys % n
# L_reg rows: off-diagonal columns + the diagonal, ascending
lists = [[] for _ in range(n)]
for r, c in zip(rows.tolist(), cols.tolist()):
    lists[r].append(c)
for i in range(n):
    lists[i].append(i)
    lists[i].sort()
# OpenBLAS chunks: width ceil(rem / threads_left)
ca, cl = [], []
a = 0
for t in range(T):
    w = -(-(n - a) // (T - t))
    ca.append(a)
    cl.append(w)
    a += w
nch = 32 * T
dsl = NT
cap = (160 * 1024 - (6 * nch + 2 * KMAX + 2 + dsl) * 8) // 8
tot = n
align = 32 * G
keep = [(cap * cl[t] // tot) // align * align for t in range(T)]
left = cap - sum(keep)
while left >= align:
    best = max((t for t in range(T) if keep[t] + align <= cl[t]), key=lambda t: cl[t] - keep[t], default=None)
    if best is None:
        break
    keep[best] += align
    left -= align
lbase = np.concatenate([[0], np.cumsum(keep)[:-1]])
zs = int(sum(keep))


def owner_tid(row):
    t = max(i for i in range(T) if row >= ca[i])
    o = row - ca[t]
    n32 = cl[t] & ~31
    inn = o < n32
    j = (o & 31) if inn else o - n32
    g = (o >> 5) % G if inn else 0
    chain = t * 32 + j
    CW = 64 // G
    return (chain // CW) * 64 + (chain % CW) + CW * g


def slot_of(x, row_owner, layout):
    """LDS double slot of p row x (None: global), the diagonal slot, the zero slot."""
    t = max(i for i in range(T) if x >= ca[i])
    o = x - ca[t]
    if o >= keep[t]:
        return None
    base = int(lbase[t]) + o
    if layout == "cur":
        return base
    if layout.startswith("rot"):  # rotate each 64-row wave slot by k rows (mod 64) per 64-block
        s = int(layout[3:])
        blk, off = divmod(o, 64)
        return int(lbase[t]) + blk * 64 + (off + s * blk) % 64
    raise ValueError(layout)


DIAG = os.environ.get("DIAG", "cur")


def diag_slot(r):
    """cur: zs + 2 + tid (the kernel); an integer s: a slot in a separate region whose
    bank is the own row's p bank + s (mod 32), one slot per row (a dense remap)."""
    if DIAG == "cur":
        return zs + 2 + owner_tid(r)
    t = max(i for i in range(T) if r >= ca[i])
    o = r - ca[t]
    own = int(lbase[t]) + o
    base = (zs + 2048) // 32 * 32 + 32
    return base + (owner_tid(r) // 32) * 32 + ((own + int(DIAG)) % 32)


ZERO = os.environ.get("ZERO", "cur")


def zero_slot(r):
    """cur: the one zero slot; an integer s: one of 32 zero slots, bank = own p bank + s."""
    if ZERO == "cur":
        return zs
    t = max(i for i in range(T) if r >= ca[i])
    own = int(lbase[t]) + r - ca[t]
    return (zs + 8192) // 32 * 32 + ((own + int(ZERO)) % 32)


def sim(layout):
    cycles = extra = insts = 0
    for t in range(T):
        L = cl[t]
        n32 = L & ~31
        for u0 in range(0, n32, 64):
            rws = [ca[t] + u0 + l for l in range(64)]
            for k in range(8):
                for grp in (rws[:32], rws[32:]):
                    addrs = []
                    for r in grp:
                        if r >= ca[t] + n32:
                            continue
                        lst = lists[r]
                        if k < len(lst):
                            c = lst[k]
                            if c == r:
                                a_ = diag_slot(r)
                            else:
                                a_ = slot_of(c, r, layout)
                                if a_ is None:
                                    a_ = 1 << 20  # global: read past the LDS (its own "bank")
                        else:
                            a_ = zero_slot(r)
                        addrs.append(a_)
                    if not addrs:
                        continue
                    banks = {}
                    for a_ in set(addrs):
                        if a_ >= (1 << 20):
                            continue
                        banks.setdefault(a_ % 32, set()).add(a_)
                    w = max((len(v) for v in banks.values()), default=1)
                    cycles += w
                    extra += w - 1
                    insts += 1
    return cycles, extra, insts


for lay in ["cur"] + sys.argv[2:]:
    c, e, i = sim(lay)
    print(f"{lay}: {i} group-accesses, {c} cycles, {e} extra (+{100.0 * e / i:.1f}% over conflict-free)")


def classify():
    """Extra cycles by the kinds of addresses sharing a bank: p (a p row), d (a
    diagonal slot), z (the zero slot)."""
    from collections import Counter

    cnt = Counter()
    for t in range(T):
        L = cl[t]
        n32 = L & ~31
        for u0 in range(0, n32, 64):
            rws = [ca[t] + u0 + l for l in range(64)]
            for k in range(8):
                for grp in (rws[:32], rws[32:]):
                    kinds = {}
                    for r in grp:
                        if r >= ca[t] + n32:
                            continue
                        lst = lists[r]
                        if k < len(lst):
                            c = lst[k]
                            if c == r:
                                a_, kd = zs + 2 + owner_tid(r), "d"
                            else:
                                a_ = slot_of(c, r, "cur")
                                if a_ is None:
                                    continue
                                kd = "p"
                        else:
                            a_, kd = zs, "z"
                        kinds[a_] = kd
                    banks = {}
                    for a_, kd in kinds.items():
                        banks.setdefault(a_ % 32, []).append(kd)
                    w = max((len(v) for v in banks.values()), default=1)
                    if w > 1:
                        worst = max(banks.values(), key=len)
                        cnt["".join(sorted(worst))] += w - 1
    for k, v in cnt.most_common(12):
        print(k, v)


if os.environ.get("CLASSIFY"):
    classify()
