"""Test configuration: package + oracle on sys.path, the `gpu` marker, golden loader.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, the
C-ABI library loading/exports); `-m gpu` tests call libgsparse.so on an
MI355X and compare with the oracle / golden vectors.
"""

import faulthandler
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnn-sparsification-research_amd")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libgsparse.so")
    # Python stacks of every thread on a fatal signal (SIGSEGV / SIGABRT inside
    # the native library), written to the real stderr even under capture
    if not faulthandler.is_enabled():
        faulthandler.enable(all_threads=True)


def golden_names(include_big=True):
    names = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz")))
    names = [n for n in names
             if n != "karate_weighted" and not n.startswith("exact_er_") and not n.startswith("bb_")]
    if not include_big:
        names = [n for n in names if n != "roman_full"]
    return names


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def exact_er_golden(name):
    """Reference calculate_effective_resistance_scores output for golden `name`
    (in the graph's own file, or exact_er_<name>.npz for the larger graphs), or None."""
    g = load_golden(name)
    if "scores_effective_resistance" in g:
        return g["scores_effective_resistance"]
    path = os.path.join(GOLDEN, f"exact_er_{name}.npz")
    if os.path.exists(path):
        return load_golden(f"exact_er_{name}")["scores_effective_resistance"]
    return None


def exact_er_names():
    return [n for n in golden_names(include_big=False) + ["karate_weighted"]
            if exact_er_golden(n) is not None]


# The reference's pinv(L + 1e-10 I) carries a 1e10/|C| direction per component
# whose rounding leaves 1e-6..5e-5 absolute noise in its R_eff (max 4.75e-5 on
# rmat10); the lifted inverse (oracle.exact_er, gs_exact_er) has none of it.
EXACT_ER_ATOL = 1e-4


def golden_features(g):
    from gsparse import graphs
    import hashlib

    if "feat_dim" not in g:
        return None
    x = graphs.features(int(g["num_nodes"]), int(g["feat_dim"]), int(g["feat_seed"]),
                        str(g["feat_kind"]))
    assert hashlib.sha256(x.tobytes()).hexdigest() == str(g["feat_sha256"]), \
        "regenerated features differ from the ones the golden vectors were made with"
    return x


def bits_equal(a, b):
    a = np.ascontiguousarray(a, dtype=np.float64)
    b = np.ascontiguousarray(b, dtype=np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))
