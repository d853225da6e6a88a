"""On-disk dataset loader (DistGNN.dataloading.load_dataset, reference load_dataset.py:5-32)
against files written exactly as the reference's dataset_preprocess.py:48-79 writes them."""
import os
import pickle

import numpy as np
import pytest
import torch

from DistGNN.dataloading import load_dataset


def _write(path, name, papers=False, bias=False, seed=0):
    rng = np.random.default_rng(seed)
    n, e, d = 50, 300, 8
    indptr = np.concatenate([[0], np.sort(rng.integers(0, e, n - 1)), [e]])
    indices = rng.integers(0, n, e)
    feats = rng.standard_normal((n, d)).astype(np.float32)
    labels = rng.integers(0, 5, n)
    torch.save(torch.from_numpy(feats).float(), os.path.join(path, "features.pt"))
    if papers:  # papers100M stores float labels with NaN for unlabelled nodes (:134-136)
        lab = labels.astype(np.float64)
        lab[::7] = np.nan
        torch.save(torch.from_numpy(lab[:, None]).float().squeeze(1),
                   os.path.join(path, "labels.pt"))
    else:
        torch.save(torch.from_numpy(labels).long(), os.path.join(path, "labels.pt"))
    torch.save(torch.from_numpy(indptr).long(), os.path.join(path, "indptr.pt"))
    torch.save(torch.from_numpy(indices).long(), os.path.join(path, "indices.pt"))
    torch.save(torch.arange(0, n, 3), os.path.join(path, "train_idx.pt"))
    if bias:
        torch.save(torch.randn(e).abs().float(), os.path.join(path, "probs.pt"))
    meta = {"dataset": name, "num_nodes": n, "num_edges": e,
            "num_classes": int(np.unique(labels).shape[0]), "feature_dim": d,
            "num_train_nodes": 17, "num_valid_nodes": 0, "num_test_nodes": 0}
    torch.save(meta, os.path.join(path, "metadata.pt"))
    return indptr, indices, feats, meta


@pytest.mark.parametrize("papers,bias", [(False, False), (True, True)])
def test_load_dataset_reference_layout(tmp_path, papers, bias):
    indptr, indices, feats, meta = _write(str(tmp_path), "ogbn-x", papers, bias)
    g, nc = load_dataset(str(tmp_path), "ogbn-x", with_feature=True, with_probs=bias)
    assert nc == meta["num_classes"]
    assert torch.equal(g["indptr"], torch.from_numpy(indptr).long())
    assert torch.equal(g["indices"], torch.from_numpy(indices).long())
    assert torch.equal(g["features"], torch.from_numpy(feats))
    assert g["labels"].dtype == (torch.float32 if papers else torch.int64)
    assert ("probs" in g) == bias
    g2, _ = load_dataset(str(tmp_path), "ogbn-x", with_feature=False)
    assert "features" not in g2 and "probs" not in g2


def test_load_dataset_name_mismatch(tmp_path):
    _write(str(tmp_path), "ogbn-products")
    with pytest.raises(AssertionError):
        load_dataset(str(tmp_path), "ogbn-papers100M")


class _Payload:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_load_dataset_refuses_pickled_code(tmp_path):
    _write(str(tmp_path), "ogbn-x")
    with open(os.path.join(str(tmp_path), "metadata.pt"), "wb") as f:
        pickle.dump({"dataset": "ogbn-x", "num_classes": _Payload()}, f)
    with pytest.raises(Exception):
        load_dataset(str(tmp_path), "ogbn-x")
