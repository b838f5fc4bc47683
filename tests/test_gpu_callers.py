"""The drop-in driven the way the reference's own callers drive it.

* scripts/nb05_roman_empire/roman_empire_gpu.py:_main_worker (:185-256): a spawn
  worker calls torch.cuda.set_device(device_str) (:209), builds
  GraphSparsifier(full_graph, device='cpu') (:213), computes the scores once
  (:219) and, for retentions 0.9 .. 0.2, sparsify / sparsify_sampled /
  sparsify_degree_aware with return_mask=True (:228-239), then edge weights as
  the min-max of all_scores[mask] (:248-256).
* src/experiments/ablation.py:AblationStudy.compute_edge_weights (:119-145): a
  NEW GraphSparsifier on every sparsified graph, scores min-max normalised and
  clipped to [0.1, 1].
Results must equal the reference's (golden vectors / the pinned oracle), and
the library context must land on the device the caller selected.
"""

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import bits_equal, golden_features, load_golden

pytestmark = pytest.mark.gpu

RETENTIONS = [0.9, 0.8, 0.6, 0.4, 0.2]


@pytest.fixture(scope="module")
def gs():
    import gsparse

    return gsparse


def _minmax_weights(all_scores, mask_np, keep_lowest):
    """roman_empire_gpu.py:248-256."""
    scores = all_scores[mask_np]
    mn, mx = scores.min(), scores.max()
    norm = (scores - mn) / (mx - mn + 1e-8)
    if keep_lowest:
        norm = 1.0 - norm
    return torch.tensor(norm, dtype=torch.float32)


@pytest.mark.parametrize("metric,variant,keep_lowest", [
    ("jaccard", "threshold", False), ("jaccard", "threshold", True),
    ("adamic_adar", "threshold", False), ("feature_cosine", "threshold", False),
    ("approx_er", "threshold", True), ("jaccard", "sampled", False),
    ("jaccard", "degree_aware", False), ("approx_er", "degree_aware", False)])
def test_roman_empire_worker_sequence(gs, metric, variant, keep_lowest):
    g = load_golden("roman2000")
    n = int(g["num_nodes"])
    x = golden_features(g)
    ei = torch.from_numpy(g["edge_index"])
    torch.cuda.set_device(torch.device("cuda:0"))  # :209
    full_graph = gs.Data(x=torch.from_numpy(x), edge_index=ei, num_nodes=n)
    sp = gs.GraphSparsifier(full_graph, device="cpu")  # :213
    assert sp._ctx.device == torch.cuda.current_device()
    all_scores = sp.compute_scores(metric)  # :219
    ref_scores = g[f"scores_{metric}"]
    assert bits_equal(all_scores, ref_scores)
    E = ei.shape[1]
    for retention in RETENTIONS:
        if variant == "sampled":
            sparse, mask = sp.sparsify_sampled(metric, retention, seed=42, return_mask=True)
            ref_mask = g[f"sampled_{metric}_{retention}"] if f"sampled_{metric}_{retention}" in g \
                else O.sampled_mask(ref_scores, E, retention, 42)
        elif variant == "degree_aware":
            sparse, mask = sp.sparsify_degree_aware(metric, retention, return_mask=True)
            key = f"degaware_{metric}_{retention}"
            ref_mask = g[key] if key in g else None  # goldens at 0.2 (and 0.5)
        else:
            sparse, mask = sp.sparsify(metric, retention, return_mask=True, keep_lowest=keep_lowest)
            ref_mask = g[f"mask_{metric}_{retention}_{int(keep_lowest)}"] \
                if f"mask_{metric}_{retention}_{int(keep_lowest)}" in g else \
                O.topk_mask(ref_scores, E, retention, keep_lowest)
        mask_np = mask.numpy()
        if ref_mask is not None:
            assert np.array_equal(mask_np, ref_mask), (retention, variant)
        assert sparse.edge_index.device.type == "cpu"
        assert sparse.edge_index.size(1) == int(mask_np.sum())
        actual_ret = float(sparse.edge_index.size(1)) / float(E)
        assert 0 < actual_ret <= 1
        w = _minmax_weights(all_scores, mask_np, keep_lowest)
        w_ref = _minmax_weights(ref_scores, mask_np, keep_lowest)
        assert torch.equal(w, w_ref)


def _compute_edge_weights(gs, data, metric, device):
    """ablation.py:119-145, verbatim semantics, on the drop-in."""
    temp_sparsifier = gs.GraphSparsifier(data, device)
    scores = temp_sparsifier.compute_scores(metric)
    scores_min = scores.min()
    scores_max = scores.max()
    if scores_max > scores_min:
        normalized = (scores - scores_min) / (scores_max - scores_min)
    else:
        normalized = np.ones_like(scores)
    normalized = np.clip(normalized, 0.1, 1.0)
    return torch.tensor(normalized, dtype=torch.float32, device=device)


@pytest.mark.parametrize("device", ["cpu", "cuda:0"])
def test_ablation_compute_edge_weights_per_sparse_graph(gs, device):
    """A fresh sparsifier per (metric, retention) sparse graph, as
    AblationStudy.run_multi_config_study drives it (ablation.py:562-599)."""
    g = load_golden("cora_like")
    n = int(g["num_nodes"])
    data = gs.Data(edge_index=torch.from_numpy(g["edge_index"]), num_nodes=n)
    study_sp = gs.GraphSparsifier(data, device)  # ablation.py:114
    for metric in ("jaccard", "adamic_adar"):
        for retention in (0.9, 0.5, 0.1):
            sparse = study_sp.sparsify(metric, retention)
            w = _compute_edge_weights(gs, sparse, metric, device)
            ei = sparse.edge_index.cpu().numpy()
            ip, ix, _ = O.canonical_csr(ei, n)
            ref = O.jaccard(ip, ix) if metric == "jaccard" else O.adamic_adar(ip, ix)
            mn, mx = ref.min(), ref.max()
            norm = (ref - mn) / (mx - mn) if mx > mn else np.ones_like(ref)
            ref_w = torch.tensor(np.clip(norm, 0.1, 1.0), dtype=torch.float32)
            assert w.device.type == torch.device(device).type
            assert torch.equal(w.cpu(), ref_w), (metric, retention)


def test_context_follows_torch_current_device(gs):
    """GraphSparsifier(..., device='cpu') after torch.cuda.set_device(k) scores on k."""
    k = torch.cuda.device_count() - 1
    torch.cuda.set_device(k)
    try:
        g = load_golden("karate_test")
        data = gs.Data(edge_index=torch.from_numpy(g["edge_index"]), num_nodes=int(g["num_nodes"]))
        sp = gs.GraphSparsifier(data, device="cpu")
        assert sp._ctx.device == k
        assert bits_equal(sp.compute_scores("jaccard"), g["scores_jaccard"])
    finally:
        torch.cuda.set_device(0)
