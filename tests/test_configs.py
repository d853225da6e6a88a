"""BASELINE configs[0] shape: arxiv-like graph, GraphSAGE fan-out [10, 10], uniform sampler.

configs[0] is the reference's CPU-runnable plumbing case (DGL's CPU sampler; DGL is not
installed here, so the CPU side is the oracle's restatement).  CPU tests run the whole
per-iteration flow of node_classification.py:219-229 on the oracle: SeedGenerator batches ->
2-hop sample + relabel -> feature / label gather, and check the structure every hop must have.
The GPU test runs the same batches through the HIP path (P2PCacheSampler, PrefetchLoader) and
requires bit-exact equality with the oracle.  Sizes are scaled down (RMAT scale 14, ef 9) so the
oracle finishes in seconds; the full arxiv-like size is a bench configuration
(tools/configs_run.sh).
"""
import numpy as np
import pytest
import torch

from DistGNN.dataloading import SeedGenerator
from DistGNN.dataloading.synthetic import rmat_csc_numpy
from oracle import oracle as O

FAN_OUT = [10, 10]


@pytest.fixture(scope="module")
def arxiv_like():
    indptr, indices = rmat_csc_numpy(14, 9, seed=20261015)
    n = indptr.size - 1
    train = torch.randperm(n, generator=torch.Generator().manual_seed(2))[: n // 10]
    feats = np.random.default_rng(11).standard_normal((n, 128)).astype(np.float32)
    labels = np.random.default_rng(12).integers(0, 40, n).astype(np.int64)
    return indptr, indices, train, feats, labels


def _batches(train, batch=256, nbatches=4):
    torch.manual_seed(1)
    out = []
    for s in SeedGenerator(train, batch, shuffle=True, drop_last=True):
        out.append(s.numpy())
        if len(out) == nbatches:
            break
    return out


def test_arxiv_config_cpu_plumbing(arxiv_like):
    indptr, indices, train, feats, labels = arxiv_like
    deg = np.diff(indptr)
    for b, seeds in enumerate(_batches(train)):
        blocks = O.node_classification_sample(seeds, indptr, indices, FAN_OUT, False,
                                              O.launch_seeds(7 + b, len(FAN_OUT)))
        assert len(blocks) == len(FAN_OUT)
        cur = seeds
        for h, (s, f, r, c) in enumerate(blocks):
            k = FAN_OUT[len(FAN_OUT) - 1 - h]
            assert np.array_equal(s, cur)
            assert np.array_equal(f[: s.size], s)            # frontier prefix == seeds
            assert np.unique(f).size == f.size
            assert r.size == np.minimum(deg[s], k).sum()     # nnz = sum min(deg, k)
            assert (r >= 0).all() and (r < s.size).all() and (c < f.size).all()
            # every pick is a neighbour of its row, no position picked twice per row
            src, dst = s[r], f[c]
            for row in np.unique(r)[:50]:
                nb = indices[indptr[s[row]]:indptr[s[row] + 1]]
                assert np.isin(dst[r == row], nb).all()
                assert src[r == row][0] == s[row]
            cur = f
        x = O.index_select(feats, cur)
        y = O.index_select(labels, seeds)
        assert np.array_equal(x, feats[cur]) and np.array_equal(y, labels[seeds])


@pytest.mark.gpu
@pytest.mark.parametrize("replace", [False, True])
@pytest.mark.parametrize("id_dtype", [torch.int64, torch.int32])
def test_arxiv_config_gpu_bit_exact(arxiv_like, replace, id_dtype):
    import dgs
    from DistGNN.dataloading import PrefetchLoader
    indptr, indices, train, feats, labels = arxiv_like
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr).to(id_dtype),
                                          torch.from_numpy(indices).to(id_dtype),
                                          torch.Tensor(), torch.arange(n), 0)
    server = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(feats), torch.arange(n), 0)
    labels_dev = torch.from_numpy(labels).cuda()
    batches = _batches(train)
    seeds_dev = [torch.from_numpy(s).to(id_dtype).cuda() for s in batches]
    # sequential loop (the reference's order) and the pipelined loader, same launch seeds
    dgs.ops._CAPI_set_random_seed(99)
    seq = []
    for s in seeds_dev:
        blocks = sampler._CAPI_sample_node_classifiction(s, FAN_OUT, replace)
        seq.append((blocks, server._CAPI_get_feature(blocks[-1][1]),
                    dgs.ops._CAPI_cuda_index_select(labels_dev, s)))
    dgs.ops._CAPI_set_random_seed(99)
    pipe = list(PrefetchLoader(sampler, seeds_dev, FAN_OUT, replace, server=server,
                               labels=labels_dev, depth=3))
    torch.cuda.synchronize()
    launch = O.launch_seeds(99, len(FAN_OUT) * len(batches))
    for b, seeds in enumerate(batches):
        exp = O.node_classification_sample(seeds, indptr, indices, FAN_OUT, replace,
                                           launch[len(FAN_OUT) * b: len(FAN_OUT) * (b + 1)])
        for got in (seq[b], pipe[b]):
            blocks, x, y = got
            for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
                assert gf.dtype == id_dtype
                assert np.array_equal(gs.cpu().numpy(), es)
                assert np.array_equal(gf.cpu().numpy(), ef)
                assert np.array_equal(gr.cpu().numpy(), er)
                assert np.array_equal(gc.cpu().numpy(), ec)
            assert np.array_equal(x.cpu().numpy(), O.index_select(feats, exp[-1][1]))
            assert np.array_equal(y.cpu().numpy(), labels[seeds])
