"""On-disk dataset loader, counterpart of python/DistGNN/dataloading/load_dataset.py:5-32.

Layout (written by the reference's dataset_preprocess.py): <path>/{metadata, labels, indptr,
indices, train_idx, features, probs}.pt.  Loaded with weights_only=True (no pickle code)."""
import os

import torch

__all__ = ["load_dataset"]


def _load(path, name):
    return torch.load(os.path.join(path, name + ".pt"), weights_only=True)


def load_dataset(path, dataset_name, with_feature=True, with_probs=False):
    meta = _load(path, "metadata")
    # the reference asserts (load_dataset.py:9)
    if meta["dataset"] != dataset_name:
        raise AssertionError(f"{path} holds {meta['dataset']}, not {dataset_name}")
    graph = {name: _load(path, name) for name in ("labels", "indptr", "indices", "train_idx")}
    if with_feature:
        graph["features"] = _load(path, "features")
    if with_probs:
        graph["probs"] = _load(path, "probs")
    return graph, meta["num_classes"]
