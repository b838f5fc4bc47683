"""libgsparse.so loads and exports exactly the C ABI declared in include/gsparse.h.

No compute calls here (no GPU needed): symbol presence, the ctypes
signature table, version/error plumbing, the host-only helper gs_er_split,
and the loud failure when no device is present.
"""

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "gsparse.h")
LIB = os.path.join(PKG, "gsparse", "libgsparse.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def built():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    return LIB


def test_header_declares_api():
    names = declared_functions()
    for must in ["gs_create", "gs_jaccard", "gs_adamic_adar", "gs_feature_cosine_f32",
                 "gs_er_solve", "gs_topk_mask", "gs_metric_backbone"]:
        assert must in names


def test_library_exports_every_declared_symbol(built):
    out = subprocess.run(["nm", "-D", "--defined-only", built], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (gs_[a-z0-9_]+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing


def test_ctypes_table_matches_header(built):
    from gsparse import _lib

    assert sorted(_lib.SIGNATURES) == declared_functions()
    L = _lib.lib(built)
    assert L.gs_api_version() == 3


def test_library_is_gfx950_code(built):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-n", built],
                         capture_output=True, text=True)
    blob = open(built, "rb").read()
    assert b"gfx950" in blob


def test_er_split_is_the_pairwise_tree(built):
    from gsparse import engine

    # numpy pairwise: n2 = n//2 - (n//2) % 8
    k = 2674
    b2 = engine.er_split(k, 2)
    n2 = k // 2 - (k // 2) % 8
    assert b2 == [0, n2, k]
    b4 = engine.er_split(k, 4)
    l2 = n2 // 2 - (n2 // 2) % 8
    r = k - n2
    r2 = r // 2 - (r // 2) % 8
    assert b4 == [0, l2, n2, n2 + r2, k]
    with pytest.raises(ValueError):
        engine.er_split(100, 2)  # a 100-wide block is a leaf: cannot split
    with pytest.raises(ValueError):
        engine.er_split(k, 3)


def test_er_split_blocks_sum_like_numpy(built):
    """sum of per-block pairwise sums combined as a tree == np.add.reduce."""
    from gsparse import engine
    import gsparse_oracle as O

    rng = np.random.default_rng(1)
    for k in [1024, 2107, 2674, 3210, 4066]:
        a = rng.standard_normal(k) ** 2
        for parts in (2, 4, 8):
            b = engine.er_split(k, parts)
            sums = [O.lib().oracle_pairwise_sum_f64(O._p(np.ascontiguousarray(a[b[i]:b[i + 1]]),
                                                         O._f64p), O.ctypes.c_int64(b[i + 1] - b[i]))
                    for i in range(parts)]
            while len(sums) > 1:
                sums = [sums[i] + sums[i + 1] for i in range(0, len(sums), 2)]
            assert 0.0 + sums[0] == np.sum(a), (k, parts)


def test_last_error_and_no_device_failure(built):
    """Without a gfx950 device, contexts fail loudly (no CPU fallback)."""
    from gsparse import _lib

    L = _lib.lib(built)
    n = ctypes.c_int(0)
    rc = L.gs_device_count(ctypes.byref(n))
    if rc == 0 and n.value > 0:
        pytest.skip("a GPU is present: covered by the gpu tests")
    with pytest.raises(_lib.GsparseUnavailable):
        _lib.Context(0)
    assert isinstance(L.gs_last_error(), bytes)
