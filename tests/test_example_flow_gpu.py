"""The reference example's data path end to end (example/graphsage/node_classification.py:
43-229 without the model): dataset from disk in the reference layout, heat-based selfish
cache plan under a memory budget (so part of the graph stays in pinned host memory), pinned
graph tensors, sampler + feature server built from the plan, then the training loop's
sample -> features -> labels -- sequential and pipelined -- checked against the CPU oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _write_dataset(path, n=4000, d=24, seed=5):
    import os
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, 40, n)
    degs[:3] = [3000, 1500, 0]  # hubs and an empty row
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, n, int(indptr[-1])).astype(np.int64)
    feats = rng.standard_normal((n, d)).astype(np.float32)
    labels = rng.integers(0, 10, n)
    torch.save(torch.from_numpy(feats).float(), os.path.join(path, "features.pt"))
    torch.save(torch.from_numpy(labels).long(), os.path.join(path, "labels.pt"))
    torch.save(torch.from_numpy(indptr).long(), os.path.join(path, "indptr.pt"))
    torch.save(torch.from_numpy(indices).long(), os.path.join(path, "indices.pt"))
    torch.save(torch.from_numpy(rng.permutation(n)[: n // 4]).long(),
               os.path.join(path, "train_idx.pt"))
    torch.save(torch.from_numpy(rng.random(indices.size).astype(np.float32) + 0.01),
               os.path.join(path, "probs.pt"))
    torch.save({"dataset": "ogbn-synth", "num_nodes": n, "num_edges": int(indptr[-1]),
                "num_classes": 10, "feature_dim": d}, os.path.join(path, "metadata.pt"))


@pytest.mark.parametrize("bias", [False, True])
def test_reference_example_data_path(tmp_path, bias):
    import dgs
    from DistGNN.cache import (get_cache_nids_selfish, get_feature_space, get_node_heat,
                               get_structure_space)
    from DistGNN.dataloading import PrefetchLoader, SeedGenerator, load_dataset
    _write_dataset(str(tmp_path))
    graph, num_classes = load_dataset(str(tmp_path), "ogbn-synth", with_probs=bias)
    assert num_classes == 10
    fan_out = [8, 5, 3] if bias else [15, 10, 5]
    probs_key = "probs" if bias else None
    train_nids = graph["train_idx"]
    sampling_heat, feature_heat = get_node_heat(
        graph["indptr"], graph["indices"], train_nids, fan_out,
        probs=graph["probs"] if bias else None)
    n = graph["indptr"].numel() - 1
    everything = (torch.sum(get_structure_space(torch.arange(n), graph, probs=probs_key))
                  + get_feature_space(graph) * n)
    budget = int(0.4 * float(everything))  # about 40 % of the graph fits
    s_nids, f_nids = get_cache_nids_selfish(graph, sampling_heat, feature_heat, budget,
                                            120.62, 480, 480, 8.32, 480, 512, probs=probs_key)
    assert 0 < s_nids.numel() < n or 0 < f_nids.numel() < n
    for key in graph:
        dgs.ops._CAPI_tensor_pin_memory(graph[key])
    probs = graph["probs"] if bias else torch.Tensor()
    # the reference requires non-empty cache lists (sampler.cc:89)
    s_nids = s_nids if s_nids.numel() else torch.tensor([0])
    f_nids = f_nids if f_nids.numel() else torch.tensor([0])
    sampler = dgs.classes.P2PCacheSampler(graph["indptr"], graph["indices"], probs, s_nids, 0)
    server = dgs.classes.P2PCacheFeatureServer(graph["features"], f_nids, 0)
    labels = graph["labels"].cuda()

    torch.manual_seed(3)
    batches = list(SeedGenerator(train_nids.cuda(), 128, shuffle=True))
    ip, ix = graph["indptr"].numpy(), graph["indices"].numpy()
    pr = graph["probs"].numpy() if bias else None
    for pipelined in (False, True):
        dgs.ops._CAPI_set_random_seed(2024)
        if pipelined:
            out = list(PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                                      depth=3))
        else:
            out = []
            for s in batches:  # node_classification.py:219-229
                blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
                x = server._CAPI_get_feature(blocks[-1][1])
                y = dgs.ops._CAPI_cuda_index_select(labels, s)
                out.append((blocks, x, y))
        torch.cuda.synchronize()
        seeds = O.launch_seeds(2024, len(fan_out) * len(batches))
        for i, (s, (blocks, x, y)) in enumerate(zip(batches, out)):
            exp = O.node_classification_sample(
                s.cpu().numpy(), ip, ix, fan_out, False,
                seeds[len(fan_out) * i:len(fan_out) * (i + 1)], probs=pr)
            for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
                assert np.array_equal(gf.cpu().numpy(), ef)
                assert np.array_equal(gr.cpu().numpy(), er)
                assert np.array_equal(gc.cpu().numpy(), ec)
            assert torch.equal(x.cpu(), graph["features"][blocks[-1][1].cpu()])
            assert torch.equal(y.cpu(), graph["labels"][s.cpu()])
