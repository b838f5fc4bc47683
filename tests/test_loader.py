"""Dataset loader (src.data stand-in): CPU-side contract and the device
canonicalisation (gs_coalesce_edges) against the oracle's to_undirected +
coalesce restatement."""

import numpy as np
import pytest
import torch

import gsparse_oracle as O
from conftest import load_golden


def test_oracle_coalesce_matches_generator_layout():
    from gsparse import graphs

    ei = graphs.roman_like(n=500, m=700, seed=3)
    assert np.array_equal(O.coalesce(ei, 500), ei)
    half = ei[:, ei[0] < ei[1]]
    assert np.array_equal(O.coalesce(half, 500), ei)


def test_missing_dataset_fails_loudly(tmp_path):
    from gsparse.loader import DatasetLoader

    with pytest.raises(FileNotFoundError, match="nothing is downloaded"):
        DatasetLoader(root=str(tmp_path)).get_dataset("cora")
    with pytest.raises(ValueError, match="unknown synthetic"):
        DatasetLoader(root=str(tmp_path)).get_dataset("synthetic-nope")


def test_src_data_exports():
    import src
    from src.data import SAFE_DATASETS, DatasetLoader
    from src.data.loader import DatasetLoader as D2

    assert DatasetLoader is D2 and src.DatasetLoader is DatasetLoader
    assert "roman_empire" in SAFE_DATASETS and "cora" in SAFE_DATASETS


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["directed_dup", "karate_test", "rmat10", "isolated", "single_edge"])
@pytest.mark.parametrize("undirected,loops", [(True, False), (True, True), (False, False), (False, True)])
def test_coalesce_vs_oracle(name, undirected, loops):
    from gsparse.loader import coalesce_edges

    g = load_golden(name)
    n = int(g["num_nodes"])
    ei = g["edge_index"]
    got = coalesce_edges(ei, n, undirected=undirected, remove_self_loops=loops)
    assert np.array_equal(got, O.coalesce(ei, n, undirected, loops))


@pytest.mark.gpu
def test_coalesce_edge_cases():
    from gsparse.loader import coalesce_edges

    assert coalesce_edges(np.zeros((2, 0), np.int64), 5).shape == (2, 0)
    loops = np.array([[1, 1, 2], [1, 1, 2]])
    assert coalesce_edges(loops, 3, remove_self_loops=True).shape == (2, 0)
    assert np.array_equal(coalesce_edges(loops, 3), [[1, 2], [1, 2]])
    with pytest.raises(ValueError, match="out of range"):
        coalesce_edges(np.array([[0], [7]]), 5)
    rng = np.random.default_rng(0)
    big = rng.integers(0, 1 << 20, size=(2, 3_000_000))
    assert np.array_equal(coalesce_edges(big, 1 << 20), O.coalesce(big, 1 << 20))


@pytest.mark.gpu
def test_loader_heterophilous_layout(tmp_path):
    """The heterophilous benchmark layout (edges [E, 2], masks [S, n]): one
    direction per edge in the file, both after loading; split_idx picks a
    column; scores on the loaded graph equal scores on the canonical list."""
    import gsparse
    from gsparse.loader import DatasetLoader

    g = load_golden("roman2000")
    n = int(g["num_nodes"])
    ei = g["edge_index"]
    half = ei[:, ei[0] < ei[1]]
    rng = np.random.default_rng(5)
    x = rng.standard_normal((n, 16)).astype(np.float32)
    y = rng.integers(0, 18, n)
    masks = rng.random((10, n)) < 0.5
    np.savez(tmp_path / "roman_empire.npz", node_features=x, node_labels=y,
             edges=half.T.copy(), train_masks=masks, val_masks=~masks, test_masks=masks)
    for split in (0, 7):
        data, nf, nc = DatasetLoader(root=str(tmp_path)).get_dataset("roman_empire", "cpu",
                                                                      split_idx=split)
        assert (nf, nc) == (16, int(y.max()) + 1) and data.num_nodes == n
        assert np.array_equal(data.edge_index.numpy(), ei)
        assert np.array_equal(data.train_mask.numpy(), masks[split])
        assert np.array_equal(data.x.numpy(), x) and np.array_equal(data.y.numpy(), y)
    sp_ = gsparse.GraphSparsifier(data, "cpu")
    assert np.array_equal(sp_.compute_scores("jaccard"), g["scores_jaccard"])


@pytest.mark.gpu
def test_loader_plain_npz_and_synthetic(tmp_path):
    from gsparse.loader import DatasetLoader

    g = load_golden("directed_dup")
    n = int(g["num_nodes"])
    np.savez(tmp_path / "mygraph.npz", edge_index=g["edge_index"], num_nodes=n)
    data, nf, nc = DatasetLoader(root=str(tmp_path)).get_dataset("mygraph")
    assert (nf, nc) == (0, 0)
    assert np.array_equal(data.edge_index.numpy(), O.coalesce(g["edge_index"], n))
    data, nf, nc = DatasetLoader(root=str(tmp_path)).get_dataset("synthetic-cora", "cpu")
    assert (data.num_nodes, nf, nc) == (2708, 1433, 7) and data.edge_index.shape[1] == 10556
    assert int(data.train_mask.sum() + data.val_mask.sum() + data.test_mask.sum()) == 2708
