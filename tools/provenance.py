"""Which code a measurement belongs to.

source_hash(): SHA-256 over the sources libgsparse.so is built from (csrc/*.hip,
*.hpp, the Makefile and include/gsparse.h), in sorted path order.  The
rocprofv3 PMC summaries under profiles/ carry it (tools/pmc_summary.py), and
bench.py only joins a summary's counter bytes to a live timing when the hash
matches the tree it is running from -- counters of other code are reported as
stale, never divided by this run's time.
"""

import glob
import hashlib
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def source_files():
    csrc = os.path.join(ROOT, "gnn-sparsification-research_amd", "csrc")
    files = glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))
    files += [os.path.join(csrc, "Makefile"), os.path.join(ROOT, "include", "gsparse.h")]
    return sorted(f for f in files if os.path.exists(f))


def source_hash() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]


def git_head() -> str | None:
    try:
        return subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"],
                              capture_output=True, text=True, timeout=10).stdout.strip() or None
    except Exception:
        return None


if __name__ == "__main__":
    print(source_hash())
