#!/usr/bin/env python3
"""Static ISA op histogram of one kernel, per phase.

usage: isa_hist.py KERNEL.s SYMBOL [OUT.json]

KERNEL.s: hipcc --cuda-device-only -S output.  The register-resident CG
(k_cg_regwide) reads the constant clock (s_memrealtime) at every phase
boundary of its iteration (lap() in gs_cg_wide.hpp), so the straight-line
code between two reads is one phase: p update | SpMV + p.q chains | finish |
r update + r.r chains | finish.  The slot loops are fully unrolled, so the
static count of a phase is its per-iteration count (the rare branches for p
rows outside LDS and rows longer than 8 entries included once each).
"""

import json
import re
import sys
from collections import Counter


def classify(op: str) -> str:
    if op.startswith("v_"):
        if re.search(r"_f64", op) and re.match(r"v_(add|mul|fma|fmac)_f64", op):
            return "valu_fp64_arith"
        if "permlane" in op or "readlane" in op or "readfirstlane" in op or "writelane" in op \
                or "_dpp" in op or "mov_b32_dpp" in op:
            return "valu_xlane"
        if "accvgpr" in op:
            return "valu_acc_move"
        if op.startswith(("v_mov", "v_cndmask")):
            return "valu_move_select"
        if op.startswith(("v_cmp", "v_cmpx")):
            return "valu_compare"
        if "_f64" in op or "cvt" in op:
            return "valu_fp64_other"
        if "sdwa" in op:
            return "valu_sdwa_decode"
        return "valu_int_addr"
    if op.startswith("ds_"):
        return "lds_read" if "read" in op or op.startswith("ds_load") else "lds_write_other"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem_load" if "load" in op else "vmem_store"
    if op.startswith("scratch_"):
        return "scratch_spill"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main() -> None:
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    phases, cur = [], Counter()
    ops = Counter()
    for l in lines[start:end]:
        t = l.strip()
        if not t or t.startswith((";", ".", "//")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op == "s_memrealtime":
            phases.append(cur)
            cur = Counter()
            continue
        cur[classify(op)] += 1
        ops[op] += 1
    phases.append(cur)
    # clock reads: tmark = wall_clock64() | column setup (r = b, b.b finish) | lap(4) |
    # p update | lap(0) | SpMV + p.q chains | lap(1) | finish | lap(2) | r update (SpMV
    # again) + r.r chains | lap(3) | finish + the column epilogue
    names = ["prologue", "column_setup", "p_update", "spmv_pq", "finish_pq", "r_update_rr",
             "finish_rr_and_rest"]
    out = {"kernel": sym, "source": path, "phases": {}}
    for i, c in enumerate(phases):
        nm = names[i] if i < len(names) else f"segment{i}"
        valu = sum(v for k, v in c.items() if k.startswith("valu"))
        out["phases"][nm] = dict(sorted(c.items()), valu_total=valu,
                                 fp64_arith_share=round(c.get("valu_fp64_arith", 0) / valu, 3) if valu else None)
    out["top_ops"] = dict(ops.most_common(40))
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(js)
    for nm, c in out["phases"].items():
        print(nm, c)


if __name__ == "__main__":
    main()
