"""Parity at BASELINE configs[3]'s shape on one GPU: the papers100M-like RMAT graph of
bench.py (scale 27, edge factor 12: N = 134,217,728, E = 1,610,612,736), degree-weighted biased
sampler (probs[e] = 1 + indeg(indices[e])) with fan-out [15, 10, 5] without
replacement, d = 128 features, everything resident in HBM, batches of 1024 seeds through
PrefetchLoader with 3 batches in flight (the bench's timed loop).

Two batches are checked bit-exact against the oracle (oracle/dgs_oracle.c): frontiers,
relabelled COO, gathered feature rows and labels.  The sampler path is the hub-split biased
kernels of rowwise_sampling_bias.cu:62-146 / rowwise_sampling_bias_p2p.cu:227-385 (rows of
degree > 2048 are split over workers), which the smaller graphs exercise on few rows only.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FAN_OUT = [15, 10, 5]
BATCH = 1024
DIM = 128


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


@pytest.fixture(scope="module")
def papers():
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr_d, indices_d = rmat_csc_torch(27, 12, seed=20261015, device=dev)
    n = indptr_d.numel() - 1
    probs = degree_probs(indptr_d, indices_d).cpu()
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats = torch.empty(n, DIM, dtype=torch.float32)
    step = 1 << 23
    for lo in range(0, n, step):  # 68.7 GB of features, generated in 4 GB slices
        hi = min(n, lo + step)
        feats[lo:hi] = torch.randn(hi - lo, DIM, generator=gen, device=dev).cpu()
    labels_d = torch.randint(0, 172, (n,), generator=gen, device=dev)
    g = torch.Generator()
    g.manual_seed(2)
    train = torch.randperm(n, generator=g)[: n // 100]
    out = dict(indptr=indptr_d.cpu(), indices=indices_d.cpu(), probs=probs, feats=feats,
               labels=labels_d, train=train, n=n)
    del indptr_d, indices_d
    torch.cuda.empty_cache()
    yield out
    out.clear()
    torch.cuda.empty_cache()


def test_papers_biased_pipeline_bit_exact(dgs, papers):
    from DistGNN.dataloading import PrefetchLoader
    P = papers
    assert P["n"] == 1 << 27 and P["indices"].numel() == (1 << 27) * 12
    sampler = dgs.classes.P2PCacheSampler(P["indptr"], P["indices"], P["probs"],
                                          torch.arange(P["n"]), 0)
    server = dgs.classes.P2PCacheFeatureServer(P["feats"], torch.arange(P["n"]), 0)
    nb = 2
    g = torch.Generator()
    g.manual_seed(5)
    perm = P["train"][torch.randperm(P["train"].numel(), generator=g)]
    batches = [perm[i * BATCH:(i + 1) * BATCH].cuda() for i in range(nb)]
    dgs.ops._CAPI_set_random_seed(61)
    got = [(blocks, x, y) for blocks, x, y in
           PrefetchLoader(sampler, batches, FAN_OUT, server=server, labels=P["labels"], depth=3)]
    torch.cuda.synchronize()
    ls = O.launch_seeds(61, len(FAN_OUT) * nb)
    ip, ix, pr = P["indptr"].numpy(), P["indices"].numpy(), P["probs"].numpy()
    labels = P["labels"].cpu().numpy()
    deg = np.diff(ip)
    hub_rows = 0
    for b, (blocks, x, y) in enumerate(got):
        seeds = batches[b].cpu().numpy()
        exp = O.node_classification_sample(seeds, ip, ix, FAN_OUT, False, ls[3 * b:3 * b + 3],
                                           probs=pr)
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
            assert np.array_equal(gs.cpu().numpy(), es)
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)
            hub_rows += int((deg[es] > 2048).sum())
        front = torch.from_numpy(exp[-1][1])
        assert torch.equal(x.cpu(), P["feats"][front])
        assert np.array_equal(y.cpu().numpy(), labels[seeds])
    assert hub_rows > 0  # the hub-split kernels ran
    del sampler, server
