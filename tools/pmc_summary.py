#!/usr/bin/env python3
"""Summarise rocprofv3 counter-collection CSVs per kernel.

usage: pmc_summary.py [--calls=N] OUT.json DIR [DIR ...]

--calls=N: the profiled command ran N bench steps (bench.py --steps S --warmup W
--box-order-steps 0: N = S + W), recorded as _meta.calls_per_run; bench.py then
divides every kernel's launches x per-launch counters of a region by N x the
region's calls per step in its live run -- exactly the kernels one timed call
launches, each weighted by its own launch count.

The summary's "_meta" records the source hash of the libgsparse sources it
profiled (tools/provenance.py) and the git HEAD; bench.py refuses to join
counters whose hash differs from the running tree's.

Each DIR is a rocprofv3 ``-d`` directory of one ``--pmc`` pass; every
``*counter_collection.csv`` under it is read.  Output: for each kernel (name
cut at the argument list), launches and the per-launch mean of each counter
(FETCH_SIZE / WRITE_SIZE are in KB as rocprofv3 reports them; on gfx950
FETCH_SIZE counts 1/2 of a wide coalesced stream -- MI355X_MICROARCH.md).
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import git_head, source_hash  # noqa: E402


def short(name: str) -> str:
    return name.split("(")[0] if not name.startswith("void rocprim") else name[:160]


def main() -> None:
    argv = sys.argv[1:]
    calls = None
    if argv and argv[0].startswith("--calls="):
        calls = int(argv.pop(0).split("=", 1)[1])
    out = argv[0]
    dirs = argv[1:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = short(row["Kernel_Name"])
                    acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, ctrs in acc.items():
        e = {}
        for c, vals in ctrs.items():
            unit = "_KB" if c in ("FETCH_SIZE", "WRITE_SIZE") else ""
            e[f"{c}{unit}_per_launch"] = round(sum(vals) / len(vals), 1)
            e["launches"] = max(e.get("launches", 0), len(vals))
        if "TCC_HIT_sum_per_launch" in e and "TCC_MISS_sum_per_launch" in e:
            h, m = e["TCC_HIT_sum_per_launch"], e["TCC_MISS_sum_per_launch"]
            e["L2_hit_rate"] = round(h / (h + m), 4) if h + m else None
        res[k] = e
    res["_meta"] = {"source_hash": source_hash(), "git_head": git_head(),
                    "passes": [os.path.basename(d.rstrip("/")) for d in dirs]}
    if calls:
        res["_meta"]["calls_per_run"] = calls
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, e in sorted(((k, e) for k, e in res.items() if k != "_meta"),
                       key=lambda kv: -kv[1].get("launches", 0))[:12]:
        print(k[:60], e)


if __name__ == "__main__":
    main()
