"""GPU tests of the drop-in boundary's contracts (not of one scorer's numbers):

* short edge-weight arrays raise the reference's IndexError -- in the Python
  shim and, for callers of the C ABI, in libgsparse itself -- instead of
  reaching the library as a short host buffer (the cause of round 1's host
  segfault in backbone_mask: a weight array with one entry per CSR entry
  for a graph with duplicate columns);
* device inputs that torch has only just produced (still queued on torch's
  current stream, possibly on recycled caching-allocator blocks) are read
  after torch has written them: Context.call orders the library's stream
  after torch's current stream.
"""

import ctypes

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal, golden_features, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


def _dup_graph():
    """Columns with duplicates and self-loops: E > nnz of the canonical CSR."""
    from gsparse import graphs

    ei = graphs.rmat(10, 8, seed=7)
    extra = ei[:, :500]
    loops = np.stack([np.arange(20), np.arange(20)])
    return np.concatenate([ei, extra, loops], axis=1).astype(np.int64), 1 << 10


def test_backbone_short_weights_raise_index_error(gs):
    from gsparse._lib import GS_HOST, Context, ptr
    from gsparse.metric_backbone import backbone_mask, pair_distances

    ei, n = _dup_graph()
    E = ei.shape[1]
    ip, ix, _ = O.canonical_csr(ei, n)
    assert len(ix) < E
    w_csr = O.scores_to_cost(O.jaccard(ip, ix), "jaccard")  # nnz entries: too short
    with pytest.raises(IndexError):
        backbone_mask(ei, n, w_csr)
    with pytest.raises(IndexError):
        pair_distances(ei, n, w_csr, [(0, 1), (2, 3)])
    data = gs.Data(edge_index=torch.from_numpy(ei), num_nodes=n)
    with pytest.raises(IndexError):
        gs.compute_metric_backbone(data, w_csr, verbose=False)
    # the C ABI checks the count itself (a caller binding it directly)
    ctx = Context()
    src, dst = np.ascontiguousarray(ei[0]), np.ascontiguousarray(ei[1])
    keep = np.zeros(E, dtype=np.uint8)
    relax = ctypes.c_int64(0)
    with pytest.raises(IndexError):
        ctx.call("gs_metric_backbone_part", n, E, ptr(src), ptr(dst), ptr(w_csr), len(w_csr),
                 GS_HOST, 1e-9, 0, 1, ptr(keep), GS_HOST, ctypes.byref(relax))
    qs = np.array([0], dtype=np.int64)
    out = np.zeros(1)
    with pytest.raises(IndexError):
        ctx.call("gs_pair_distances", n, E, ptr(src), ptr(dst), ptr(w_csr), len(w_csr), GS_HOST,
                 1, ptr(qs), ptr(qs), ptr(out))
    # one weight per column works and matches the oracle
    rows = np.repeat(np.arange(n), np.diff(ip))
    pos = np.searchsorted(rows.astype(np.int64) * n + ix, ei[0] * n + ei[1])
    w = w_csr[pos]
    assert np.array_equal(backbone_mask(ei, n, w), O.metric_backbone(ei, n, w))


def test_hub_graph_multi_source_regression(gs, monkeypatch):
    """The exact configuration of round 1's host segfault (2 sources per
    workgroup, 256 threads, certificates off, the duplicate-column hub graph),
    now with one weight per column."""
    from test_gpu_parity import _column_costs, _hub_graph
    from gsparse.metric_backbone import backbone_mask

    ei, n = _hub_graph()
    w = _column_costs(ei, n)
    assert len(w) == ei.shape[1]
    monkeypatch.setenv("GSPARSE_BB_LANDMARKS", "0")
    monkeypatch.setenv("GSPARSE_BB_THREADS", "256")
    monkeypatch.setenv("GSPARSE_BB_MULTI", "2")
    multi = backbone_mask(ei, n, w)
    monkeypatch.setenv("GSPARSE_BB_MULTI", "1")
    single = backbone_mask(ei, n, w)
    assert np.array_equal(multi, single)
    monkeypatch.delenv("GSPARSE_BB_LANDMARKS")
    assert np.array_equal(backbone_mask(ei, n, w), single)


def _busy(dev):
    """Queue ~100 ms of work on torch's current stream."""
    a = torch.randn(4096, 4096, device=dev)
    for _ in range(40):
        a = torch.tanh(a @ a * 1e-4)
    return a


@pytest.mark.parametrize("side_stream", [False, True])
def test_inputs_just_produced_by_torch(gs, side_stream):
    g = load_golden("roman2000")
    x = golden_features(g)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev) if side_stream else torch.cuda.current_stream(dev)
    with torch.cuda.stream(s):
        for _ in range(2):
            a = _busy(dev)
            zero = (a[0, 0] * 0).to(torch.int32)
            # int32 edge_index converted by core.py (.to(torch.int64)) after the busy work
            ei32 = torch.from_numpy(g["edge_index"]).to(dev).to(torch.int32) + zero
            xd = torch.from_numpy(x.astype(np.float64)).to(dev).float() + zero.float()
            data = gs.Data(edge_index=ei32, x=xd, num_nodes=int(g["num_nodes"]))
            data.edge_index = ei32.to(torch.int64)
            sp_ = gs.GraphSparsifier(data, "cuda:0")
            assert bits_equal(sp_.compute_scores("jaccard"), g["scores_jaccard"])
            a = _busy(dev)
            data.x = xd + a[0, 0].float() * 0
            assert bits_equal(sp_.compute_scores("feature_cosine"), g["scores_feature_cosine"])
            del a, xd, ei32, data, sp_


def test_backbone_stages_device_inputs_checked(gs):
    """BackboneStages with device tensors of other dtypes -- an int32
    edge_index and float32 weights are cast (the library reads 8 B per column), giving
    the int64 / float64 mask; an output buffer of the wrong dtype, size or device is
    refused before the library writes into it."""
    from gsparse._lib import Context
    from gsparse.metric_backbone import BackboneStages, backbone_mask

    g = load_golden("rmat10")
    ei, n = g["edge_index"], int(g["num_nodes"])
    w = g["cost_jaccard"] if "cost_jaccard" in g else np.linspace(0.1, 2.0, ei.shape[1])
    ref = backbone_mask(ei, n, w)
    dev = torch.device("cuda", 0)
    E = ei.shape[1]
    for ei_t, w_t in ((torch.from_numpy(ei).to(dev).to(torch.int32), torch.from_numpy(w).to(dev).float()),
                      (torch.from_numpy(ei).to(dev), torch.from_numpy(w).to(dev))):
        st = BackboneStages(Context(0))
        w32 = w_t.double() if w_t.dtype == torch.float32 else w_t
        exp = backbone_mask(ei, n, w32.cpu().numpy())  # float32 weights: the rounded values
        st.begin(ei_t, n, w_t, 1e-9, 0, 1)
        st.certify(0, 1)
        nb = st.plan()
        st.search(0, nb, 0, 1)
        keep = torch.zeros(E, dtype=torch.uint8, device=dev)
        st.finish(keep)
        assert np.array_equal(keep.cpu().numpy().astype(bool), exp)
    assert np.array_equal(exp, ref)
    st = BackboneStages(Context(0))
    st.begin(torch.from_numpy(ei).to(dev), n, torch.from_numpy(w).to(dev), 1e-9, 0, 1)
    with pytest.raises(TypeError):
        st.state_io(torch.zeros(E, dtype=torch.int32, device=dev), out=True)
    with pytest.raises(ValueError):
        st.state_io(torch.zeros(E - 1, dtype=torch.uint8, device=dev), out=True)
    with pytest.raises(TypeError):
        st.pair_part(ei, n, w, 1e-9, 0, 1, np.zeros(E, dtype=np.int64))
    with pytest.raises(ValueError):
        st.pair_part(ei, n, w, 1e-9, 0, 1, np.zeros(E - 1, dtype=np.uint8))
