"""Parity at BASELINE configs[1]'s full size: the products-like RMAT graph of bench.py (scale 21,
edge factor 59: N = 2,097,152, E = 123,731,968), whole graph + d = 100 features in HBM, batches
of 1024 seeds with fan-out [15, 10, 5] run through PrefetchLoader with 3 batches in flight
(the bench's timed loop).

- bit-exact against the oracle (oracle/dgs_oracle.c via oracle.py) for a few batches, uniform
  and degree-weighted biased: frontiers, relabelled COO, gathered features and labels;
- with replacement (uniform and biased), two batches each, bit-exact;
- configs[4]'s RMAT-1B shape (scale 26, edge factor 16: 67 M nodes, 1.07 B edges, d = 256): two
  pipelined batches bit-exact, uniform and biased, features included;
- size-independent properties over many batches: every frontier starts with its seeds and has
  no repeated id, rows index the hop's seeds and columns its frontier, every sampled pair is an
  edge of the graph, and (without replacement) each row keeps min(deg, k) picks.
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

FAN_OUT = [15, 10, 5]
BATCH = 1024


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


@pytest.fixture(scope="module")
def products():
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr_d, indices_d = rmat_csc_torch(21, 59, seed=20261015, device=dev)
    n = indptr_d.numel() - 1
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats_d = torch.randn(n, 100, generator=gen, device=dev)
    labels_d = torch.randint(0, 47, (n,), generator=gen, device=dev)
    probs = degree_probs(indptr_d, indices_d).cpu()
    g = torch.Generator()
    g.manual_seed(2)
    train = torch.randperm(n, generator=g)[: n // 10]
    out = dict(indptr=indptr_d.cpu(), indices=indices_d.cpu(), probs=probs, feats=feats_d.cpu(),
               labels=labels_d, train=train, n=n)
    del indptr_d, indices_d, feats_d
    torch.cuda.empty_cache()
    return out


def _batches(train, nb, seed):
    g = torch.Generator()
    g.manual_seed(seed)
    perm = train[torch.randperm(train.numel(), generator=g)]
    return [perm[i * BATCH:(i + 1) * BATCH].cuda() for i in range(nb)]


def _services(dgs, P, bias):
    sampler = dgs.classes.P2PCacheSampler(P["indptr"], P["indices"],
                                          P["probs"] if bias else torch.Tensor(),
                                          torch.arange(P["n"]), 0)
    server = dgs.classes.P2PCacheFeatureServer(P["feats"], torch.arange(P["n"]), 0)
    return sampler, server


def _pipelined(dgs, sampler, server, labels, batches, replace=False):
    from DistGNN.dataloading import PrefetchLoader
    out = []
    for blocks, x, y in PrefetchLoader(sampler, batches, FAN_OUT, replace=replace, server=server,
                                       labels=labels, depth=3):
        out.append((blocks, x, y))
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("bias", [False, True])
def test_products_pipeline_bit_exact(dgs, products, bias):
    P = products
    sampler, server = _services(dgs, P, bias)
    nb = 8 if not bias else 4
    batches = _batches(P["train"], nb, seed=1)
    dgs.ops._CAPI_set_random_seed(2026)
    got = _pipelined(dgs, sampler, server, P["labels"], batches)
    ls = O.launch_seeds(2026, len(FAN_OUT) * nb)
    ip, ix = P["indptr"].numpy(), P["indices"].numpy()
    pr = P["probs"].numpy() if bias else None
    feats, labels = P["feats"].numpy(), P["labels"].cpu().numpy()
    for b, (blocks, x, y) in enumerate(got):
        seeds = batches[b].cpu().numpy()
        exp = O.node_classification_sample(seeds, ip, ix, FAN_OUT, False,
                                           ls[3 * b:3 * b + 3], probs=pr)
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
            assert np.array_equal(gs.cpu().numpy(), es)
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)
        front = exp[-1][1]
        assert np.array_equal(x.cpu().numpy().view(np.uint32), feats[front].view(np.uint32))
        assert np.array_equal(y.cpu().numpy(), labels[seeds])


@pytest.mark.parametrize("bias", [False, True])
def test_products_with_replacement_bit_exact(dgs, products, bias):
    """K3 (uniform) and K6 (biased CDF + upper_bound) with replacement at full size."""
    P = products
    sampler, server = _services(dgs, P, bias)
    batches = _batches(P["train"], 2, seed=9)
    dgs.ops._CAPI_set_random_seed(404)
    got = _pipelined(dgs, sampler, server, P["labels"], batches, replace=True)
    ls = O.launch_seeds(404, len(FAN_OUT) * 2)
    ip, ix = P["indptr"].numpy(), P["indices"].numpy()
    pr = P["probs"].numpy() if bias else None
    for b, (blocks, x, y) in enumerate(got):
        exp = O.node_classification_sample(batches[b].cpu().numpy(), ip, ix, FAN_OUT, True,
                                           ls[3 * b:3 * b + 3], probs=pr)
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)


def test_products_pipeline_properties(dgs, products):
    P = products
    sampler, server = _services(dgs, P, False)
    nb = 120
    batches = _batches(P["train"], nb, seed=3)
    dgs.ops._CAPI_set_random_seed(7)
    got = _pipelined(dgs, sampler, server, P["labels"], batches)
    dev = torch.device("cuda", 0)
    indptr = P["indptr"].to(dev)
    indices = P["indices"].to(dev)
    n = P["n"]
    deg = indptr[1:] - indptr[:-1]
    # every edge (dst v, src u) of the CSC as the key v * n + u, sorted, for membership tests
    dst = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    keys = torch.sort(dst * n + indices).values
    del dst
    feats = P["feats"].to(dev)
    total = 0
    for b, (blocks, x, y) in enumerate(got):
        seeds = batches[b]
        assert torch.equal(blocks[0][0], seeds)
        for h, (s, f, r, c) in enumerate(blocks):
            S, U = s.numel(), f.numel()
            assert torch.equal(f[:S], s)  # frontier = seeds first, then new ids
            assert torch.unique(f).numel() == U
            assert int(r.min()) >= 0 and int(r.max()) < S
            assert int(c.min()) >= 0 and int(c.max()) < U
            k = FAN_OUT[len(FAN_OUT) - 1 - h]  # the seed hop uses fan_out[-1]
            want = torch.minimum(deg[s], torch.full_like(s, k))
            assert torch.equal(torch.bincount(r, minlength=S), want)
            q = s[r] * n + f[c]
            pos = torch.searchsorted(keys, q).clamp(max=keys.numel() - 1)
            assert torch.equal(keys[pos], q)  # every sampled pair is an edge
            total += r.numel()
            if h + 1 < len(blocks):
                assert torch.equal(blocks[h + 1][0], f)
        assert torch.equal(x, feats[blocks[-1][1]])
        assert torch.equal(y, P["labels"][seeds])
    assert total > nb * 100_000  # ~340 K sampled edges per batch on this graph


@pytest.fixture(scope="module")
def rmat1b():
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr_d, indices_d = rmat_csc_torch(26, 16, seed=20261015, device=dev)
    n = indptr_d.numel() - 1
    probs = degree_probs(indptr_d, indices_d).cpu()
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats = torch.empty(n, 256, dtype=torch.float32)
    step = 1 << 22
    for lo in range(0, n, step):  # 68.7 GB of features, generated in 4 GB slices
        hi = min(n, lo + step)
        feats[lo:hi] = torch.randn(hi - lo, 256, generator=gen, device=dev).cpu()
    labels_d = torch.randint(0, 47, (n,), generator=gen, device=dev)
    g = torch.Generator()
    g.manual_seed(2)
    train = torch.randperm(n, generator=g)[: n // 10]
    out = dict(indptr=indptr_d.cpu(), indices=indices_d.cpu(), probs=probs, feats=feats,
               labels=labels_d, train=train, n=n)
    del indptr_d, indices_d
    torch.cuda.empty_cache()
    yield out
    out.clear()
    torch.cuda.empty_cache()


@pytest.mark.parametrize("bias", [False, True])
def test_rmat1b_pipeline_bit_exact(dgs, rmat1b, bias):
    P = rmat1b
    sampler = dgs.classes.P2PCacheSampler(P["indptr"], P["indices"],
                                          P["probs"] if bias else torch.Tensor(),
                                          torch.arange(P["n"]), 0)
    server = dgs.classes.P2PCacheFeatureServer(P["feats"], torch.arange(P["n"]), 0) \
        if not bias else None
    nb = 2
    batches = _batches(P["train"], nb, seed=5)
    dgs.ops._CAPI_set_random_seed(31)
    got = _pipelined(dgs, sampler, server, P["labels"], batches)
    ls = O.launch_seeds(31, len(FAN_OUT) * nb)
    ip, ix = P["indptr"].numpy(), P["indices"].numpy()
    pr = P["probs"].numpy() if bias else None
    for b, (blocks, x, y) in enumerate(got):
        seeds = batches[b].cpu().numpy()
        exp = O.node_classification_sample(seeds, ip, ix, FAN_OUT, False,
                                           ls[3 * b:3 * b + 3], probs=pr)
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)
        if server is not None:
            front = torch.from_numpy(exp[-1][1])
            assert torch.equal(x.cpu(), P["feats"][front])
    del sampler, server
