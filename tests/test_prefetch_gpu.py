"""Pipelined batch preparation (DistGNN.dataloading.PrefetchLoader) and the per-stream sampling
contexts under it: several batches in flight on separate streams over one sampler must give
exactly the sequential loop's blocks, features and labels (bit-exact), and the seeded entry
point must reproduce the engine-drawn call."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


def _graph(seed=3, n=3000):
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, 60, n)
    degs[:4] = [0, 5, 4000, 700]  # empty row, deg < k, uniform hubs on both modulo paths
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, n, int(indptr[-1])).astype(np.int64)
    probs = (rng.random(indices.size) + 0.01).astype(np.float32)
    return indptr, indices, probs


def _services(dgs, bias, id_dtype=torch.int64, dim=33):
    indptr, indices, probs = _graph()
    n = indptr.size - 1
    ip, ix = torch.from_numpy(indptr).to(id_dtype), torch.from_numpy(indices).to(id_dtype)
    pr = torch.from_numpy(probs) if bias else torch.Tensor()
    sampler = dgs.classes.P2PCacheSampler(ip, ix, pr, torch.arange(0, n, 3), 0)
    feats = torch.arange(n * dim, dtype=torch.float32).reshape(n, dim)
    server = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(1, n, 2), 0)
    labels = torch.randint(0, 40, (n,), generator=torch.Generator().manual_seed(0)).cuda()
    return (indptr, indices, probs), sampler, server, labels, feats


def _batches(n, nb=12, bsz=64, id_dtype=torch.int64):
    g = torch.Generator().manual_seed(9)
    out = [torch.randint(0, n, (bsz,), generator=g) for _ in range(nb)]
    out[min(1, nb - 1)][:4] = torch.tensor([0, 1, 2, 3])  # the special rows in one batch
    return [b.to(id_dtype).cuda() for b in out]


def _sequential(dgs, sampler, server, labels, batches, fan_out, replace=False):
    out = []
    for s in batches:
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, replace)
        x = server._CAPI_get_feature(blocks[-1][1])
        y = dgs.ops._CAPI_cuda_index_select(labels, s)
        out.append((blocks, x, y))
    return out


def _same(a, b):
    (ba, xa, ya), (bb, xb, yb) = a, b
    assert len(ba) == len(bb)
    for ta, tb in zip(ba, bb):
        for u, v in zip(ta, tb):
            assert u.dtype == v.dtype and torch.equal(u, v)
    assert torch.equal(xa, xb) and torch.equal(ya, yb)


@pytest.mark.parametrize("depth", [1, 2, 4])
@pytest.mark.parametrize("bias", [False, True])
def test_prefetch_matches_sequential(dgs, depth, bias):
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, bias)
    fan_out = [8, 5, 3] if bias else [15, 10, 5]
    batches = _batches(labels.numel())
    dgs.ops._CAPI_set_random_seed(77)
    exp = _sequential(dgs, sampler, server, labels, batches, fan_out)
    dgs.ops._CAPI_set_random_seed(77)
    got = list(PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                              depth=depth))
    torch.cuda.synchronize()
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        _same(g, e)


@pytest.mark.parametrize("bias", [False, True])
def test_prefetch_with_replacement(dgs, bias):
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, bias)
    fan_out = [6, 4, 3]
    batches = _batches(labels.numel(), nb=7)
    dgs.ops._CAPI_set_random_seed(31)
    exp = _sequential(dgs, sampler, server, labels, batches, fan_out, replace=True)
    dgs.ops._CAPI_set_random_seed(31)
    got = list(PrefetchLoader(sampler, batches, fan_out, replace=True, server=server,
                              labels=labels, depth=3))
    torch.cuda.synchronize()
    for g, e in zip(got, exp):
        _same(g, e)


def test_prefetch_int32_ids_and_oracle(dgs):
    """int32 graph ids (cast outputs), and the pipelined blocks against the CPU oracle."""
    from DistGNN.dataloading import PrefetchLoader
    (indptr, indices, _), sampler, server, labels, feats = _services(dgs, False, torch.int32)
    fan_out = [10, 4]
    batches = _batches(labels.numel(), nb=6, id_dtype=torch.int32)
    dgs.ops._CAPI_set_random_seed(5)
    got = list(PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels, depth=3))
    allseeds = O.launch_seeds(5, 2 * len(batches))  # the engine's sequence, 2 per batch
    for i, (s, (blocks, x, y)) in enumerate(zip(batches, got)):
        exp = O.node_classification_sample(s.cpu().numpy().astype(np.int64), indptr, indices,
                                           fan_out, False, allseeds[2 * i:2 * i + 2])
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(blocks, exp):
            assert gf.dtype == torch.int32
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)
        assert torch.equal(x.cpu(), feats[blocks[-1][1].long().cpu()])
        assert torch.equal(y, labels[s.long()])


def test_seeded_call_equals_engine_call(dgs):
    _, sampler, _, labels, _ = _services(dgs, False)
    s = _batches(labels.numel(), nb=1)[0]
    dgs.ops._CAPI_set_random_seed(123)
    a = sampler._CAPI_sample_node_classifiction(s, [15, 10, 5], False)
    dgs.ops._CAPI_set_random_seed(123)
    ls = dgs.ops.draw_launch_seeds(3)
    b = sampler._sample_seeded(s, [15, 10, 5], False, ls)
    for ta, tb in zip(a, b):
        for u, v in zip(ta, tb):
            assert torch.equal(u, v)
    with pytest.raises(RuntimeError):
        sampler._sample_seeded(s, [15, 10, 5], False, ls[:2])


def test_concurrent_streams_share_one_sampler(dgs):
    """Two streams sampling at once through one sampler (no loader): each stream's results
    equal the same seeded call made alone."""
    import threading
    _, sampler, _, labels, _ = _services(dgs, False)
    batches = _batches(labels.numel(), nb=8)
    seeds = [dgs.ops.draw_launch_seeds(3) for _ in batches]
    exp = [sampler._sample_seeded(s, [15, 10, 5], False, ls) for s, ls in zip(batches, seeds)]
    torch.cuda.synchronize()
    got = [None] * len(batches)

    def run(w):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            for i in range(w, len(batches), 2):
                got[i] = sampler._sample_seeded(batches[i], [15, 10, 5], False, seeds[i])
            st.synchronize()

    ths = [threading.Thread(target=run, args=(w,)) for w in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for g, e in zip(got, exp):
        for ta, tb in zip(g, e):
            for u, v in zip(ta, tb):
                assert torch.equal(u, v)


def test_prefetch_propagates_errors_in_order(dgs):
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, False)
    n = labels.numel()
    batches = _batches(n, nb=5)
    batches[3] = batches[3].clone()
    batches[3][0] = n + 5  # outside [0, num_nodes)
    it = PrefetchLoader(sampler, batches, [5, 5], server=server, depth=2)
    for _ in range(3):
        next(it)
    with pytest.raises(RuntimeError, match="outside"):
        next(it)


@pytest.mark.parametrize("host_async", [False, True])
def test_begin_end_protocol(dgs, host_async):
    """One outstanding call per stream; a second begin, or an end without a begin, raises and
    leaves the context usable."""
    _, sampler, _, labels, _ = _services(dgs, False)
    s = _batches(labels.numel(), nb=1)[0]
    dgs.ops._CAPI_set_random_seed(11)
    exp = sampler._CAPI_sample_node_classifiction(s, [10, 5], False)
    dgs.ops._CAPI_set_random_seed(11)
    p = sampler._sample_begin(s, [10, 5], False, host_async=host_async)
    with pytest.raises(RuntimeError, match="not been ended"):
        sampler._sample_begin(s, [10, 5], False, host_async=host_async)
    got = p.result()
    for ta, tb in zip(got, exp):
        for u, v in zip(ta, tb):
            assert torch.equal(u, v)
    from dgs._lib import c_i64, lib
    sizes = (c_i64 * 6)()
    assert lib.dgs_sampler_sample_end(sampler._h, 2, sizes,
                                      dgs._lib.stream_ptr(torch.device("cuda", 0))) != 0
    again = sampler._CAPI_sample_node_classifiction(s, [10, 5], False)
    assert again[0][1].numel() > 0


def test_prefetch_outputs_survive_caller_memory_reuse(dgs):
    """A caller that drops each batch at once and fills freshly allocated memory on its stream
    (a training step recycling the blocks) must not corrupt the batches still in flight, and a
    loader closed mid-way leaves the memory it dropped safe to reuse."""
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, False)
    fan_out = [15, 10, 5]
    batches = _batches(labels.numel(), nb=12)
    dgs.ops._CAPI_set_random_seed(5)
    exp = _sequential(dgs, sampler, server, labels, batches, fan_out)
    dgs.ops._CAPI_set_random_seed(5)
    kept = []
    for blocks, x, y in PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                                       depth=3):
        kept.append(([tuple(t.clone() for t in b) for b in blocks], x.clone(), y.clone()))
        del blocks, x, y
        junk = torch.full((1 << 22,), -7, dtype=torch.int64, device="cuda")  # reuses freed blocks
        junk.add_(1)
        del junk
    torch.cuda.synchronize()
    for a, b in zip(kept, exp):
        _same(a, b)
    # closed after two of twelve batches: the in-flight calls end, their memory is recycled
    loader = iter(PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels, depth=3))
    next(loader)
    next(loader)
    loader.close()
    junk = torch.full((1 << 22,), 3, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    assert int(junk.min()) == 3 and int(junk.max()) == 3


def test_two_live_loaders_on_one_sampler(dgs):
    """Two loaders over one sampler consumed in lock step (zip): each has its own streams, so
    neither hits the other's outstanding call, and each batch equals the seeded sequential call
    with the launch seeds of its submission slot (loader A fills its `depth` slots, then B, then
    they alternate one batch each)."""
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, False)
    fan_out = [15, 10, 5]
    a_b, b_b = _batches(labels.numel(), nb=6), _batches(labels.numel(), nb=12)[6:]
    depth = 3
    dgs.ops._CAPI_set_random_seed(41)
    got = list(zip(PrefetchLoader(sampler, a_b, fan_out, server=server, labels=labels,
                                  depth=depth),
                   PrefetchLoader(sampler, b_b, fan_out, server=server, labels=labels,
                                  depth=depth)))
    torch.cuda.synchronize()
    order = [("a", i) for i in range(depth)] + [("b", i) for i in range(depth)]
    for i in range(depth, len(a_b)):
        order += [("a", i), ("b", i)]
    dgs.ops._CAPI_set_random_seed(41)
    seeds = {slot: dgs.ops.draw_launch_seeds(len(fan_out)) for slot in order}
    for i, (ga, gb) in enumerate(got):
        for which, batches, g in (("a", a_b, ga), ("b", b_b, gb)):
            s = batches[i]
            blocks = sampler._sample_seeded(s, fan_out, False, seeds[(which, i)])
            exp = (blocks, server._CAPI_get_feature(blocks[-1][1]),
                   dgs.ops._CAPI_cuda_index_select(labels, s))
            _same(g, exp)


def test_loader_streams_are_returned(dgs):
    """A finished or closed loader gives its streams back; a live one keeps them."""
    from DistGNN.dataloading import PrefetchLoader
    from DistGNN.dataloading import prefetch as P
    _, sampler, server, labels, _ = _services(dgs, False)
    batches = _batches(labels.numel(), nb=4)
    first = PrefetchLoader(sampler, batches, [5, 5], server=server, depth=2)
    second = PrefetchLoader(sampler, batches, [5, 5], server=server, depth=2)
    assert not {s.cuda_stream for s in first._streams} & {s.cuda_stream for s in second._streams}
    list(first)
    assert not first._streams
    second.close()
    dev = torch.device("cuda", torch.cuda.current_device())
    assert len(P._FREE_STREAMS[dev]) >= 4


@pytest.mark.parametrize("kind", ["int64", "int32", "float32", "int64x3", "no_server",
                                  "zero_width"])
def test_prefetch_label_rows(dgs, kind):
    """The label gather rides in the feature gather's launch for 4- and 8-byte label rows
    (dgs_loader_gather); wider rows, server-less loaders and zero-width feature matrices (no
    feature launch to ride in) take the separate gather."""
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, feats = _services(dgs, False)
    base = labels.long()
    lab = {"int64": base, "int32": base.int(), "float32": base.float() * 0.5 + 0.25,
           "int64x3": torch.stack([base, base * 3, -base], 1),
           "no_server": base, "zero_width": base}[kind]
    srv = None if kind == "no_server" else server
    if kind == "zero_width":
        feats = torch.empty((feats.shape[0], 0), dtype=torch.float32)
        srv = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(1, feats.shape[0], 2), 0)
    batches = _batches(base.numel(), nb=6)
    got = list(PrefetchLoader(sampler, batches, [5, 3], server=srv, labels=lab, depth=3))
    torch.cuda.synchronize()
    lab_d = lab.to(batches[0].device)
    for s, (blocks, x, y) in zip(batches, got):
        assert y.dtype == lab.dtype and torch.equal(y, lab_d[s.long()])
        if srv is None:
            assert x is None
        else:
            assert torch.equal(x.cpu(), feats[blocks[-1][1].long().cpu()])


def test_prefetch_submit_error_surfaces_once(dgs):
    """A batch that cannot be submitted (host seeds) fails the call that would submit it, after
    the batches before it came out; the loader can still be closed."""
    from DistGNN.dataloading import PrefetchLoader
    _, sampler, server, labels, _ = _services(dgs, False)
    batches = _batches(labels.numel(), nb=5)
    batches[3] = batches[3].cpu()
    it = PrefetchLoader(sampler, batches, [5, 5], server=server, depth=2)
    for _ in range(2):
        next(it)
    with pytest.raises(RuntimeError):  # the call that submits batch 3
        next(it)
    it.close()
    with pytest.raises(StopIteration):
        next(it)


def test_prefetch_wide_gather_dropped_at_once(dgs):
    """The hazard behind the round-3 N = 2 fault: the caller drops x while its (long, wide)
    gather is still running, and the next batches' sample outputs must not land in that memory
    before the gather is done.  Feature rows of 16 KiB make every gather tens of MB; the
    batches must equal the sequential loop's, with no id left unwritten (-1)."""
    from DistGNN.dataloading import PrefetchLoader
    indptr, indices, _ = _graph()
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(n), 0)
    dim = 4096
    feats = torch.randn(n, dim, generator=torch.Generator().manual_seed(4))
    server = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(n), 0)
    labels = torch.randint(0, 40, (n,), generator=torch.Generator().manual_seed(0)).cuda()
    fan_out = [15, 10, 5]
    batches = _batches(n, nb=24, bsz=128)
    dgs.ops._CAPI_set_random_seed(13)
    exp = []
    for s in batches:
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        exp.append(([tuple(t.cpu() for t in b) for b in blocks],
                    float(server._CAPI_get_feature(blocks[-1][1]).double().sum())))
    dgs.ops._CAPI_set_random_seed(13)
    got = []
    for blocks, x, _ in PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                                       depth=3):
        got.append(([tuple(t.cpu() for t in b) for b in blocks], float(x.double().sum())))
        del blocks, x  # x's gather may still run: its memory goes back to the pool at once
    torch.cuda.synchronize()
    assert len(got) == len(exp)
    for (gb, gx), (eb, ex) in zip(got, exp):
        assert gx == ex
        for tg, te in zip(gb, eb):
            for u, v in zip(tg, te):
                assert torch.equal(u, v)
            assert int(tg[3].min()) >= 0 if tg[3].numel() else True


def _bad_id_graph(dgs, bias):
    """64 nodes of degree 3, node v -> (3v, 3v+1, 3v+2) mod 64, except that node 0's second
    neighbour is 69 (outside [0, 64): the reference would read out of bounds).  Seed 0 meets it
    at the first hop; seed 21 (neighbours 63, 0, 1) only at the second."""
    n = 64
    indptr = torch.arange(0, 3 * n + 1, 3, dtype=torch.int64)
    indices = torch.arange(3 * n, dtype=torch.int64) % n
    indices[1] = n + 5
    probs = torch.ones(indices.numel()) if bias else torch.Tensor()
    return dgs.classes.P2PCacheSampler(indptr, indices, probs, torch.arange(n), 0), n


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("case", ["first_hop", "last_hop_of_one", "last_hop_of_two",
                                  "middle_hop"])
def test_out_of_range_neighbour_id_raises(dgs, bias, case):
    """A sampled neighbour id outside [0, num_nodes) makes the call that sampled it raise --
    also when it is first met at the call's last hop (each hop's count pass checks the ids
    before the sizes are published) -- with the hop that met it; the id stays out of the
    frontier, and the same sampler's next call, which does not reach it, returns normally
    (the flag is tagged by call: nothing sticks to the stream context)."""
    sampler, n = _bad_id_graph(dgs, bias)
    seeds, fan_out, hop = {"first_hop": ([0, 7], [4, 4], 0),
                           "last_hop_of_one": ([0, 7], [4], 0),
                           "last_hop_of_two": ([21], [4, 4], 1),
                           "middle_hop": ([21], [4, 4, 4], 1)}[case]
    s = torch.tensor(seeds, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match=f"outside \\[0, num_nodes\\).*hop {hop} .*id {n + 5}"):
        sampler._CAPI_sample_node_classifiction(s, fan_out, False)
    for _ in range(2):  # usable afterwards, on the same stream context
        blocks = sampler._CAPI_sample_node_classifiction(
            torch.tensor([9, 10], dtype=torch.int64, device="cuda"), fan_out, False)
        assert int(blocks[-1][1].max()) < n and int(blocks[-1][3].min()) >= 0


def test_out_of_range_id_raises_in_its_own_batch(dgs):
    """Pipelined: the batch whose last hop meets the bad id raises when it is handed out, not a
    later batch (round 3: the last hop's flag surfaced at the stream's next call)."""
    from DistGNN.dataloading import PrefetchLoader
    sampler, n = _bad_id_graph(dgs, False)
    mk = lambda ids: torch.tensor(ids, dtype=torch.int64, device="cuda")  # noqa: E731
    ld = iter(PrefetchLoader(sampler, [mk([9]), mk([0, 7]), mk([10]), mk([11])], [4], depth=3))
    blocks, _, _ = next(ld)
    assert int(blocks[0][1].max()) < n
    with pytest.raises(RuntimeError, match="outside \\[0, num_nodes\\)"):
        next(ld)


def test_sampler_contexts_are_bounded(dgs):
    """A caller that samples under 32 fresh streams (e.g. a new torch.cuda.Stream per call):
    the sampler keeps at most 8 per-stream contexts (the least recently used idle one is evicted
    after its last kernels finished), device memory stays bounded, and every call on every
    stream is bit-exact against the same call on the default stream."""
    from DistGNN.dataloading.synthetic import rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(20, 4, seed=5)  # 2^20 nodes: 16 MB of relabel tables
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(indptr.size - 1), 0)
    fan_out, ls = [15, 10, 5], [11, 22, 33]
    seeds = torch.randint(0, indptr.size - 1, (512,), generator=torch.Generator().manual_seed(1))
    seeds = seeds.cuda()
    exp = sampler._sample_seeded(seeds, fan_out, False, ls)
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free0 = torch.cuda.mem_get_info()[0]
    per_ctx = None
    streams = [torch.cuda.Stream() for _ in range(32)]
    assert len({s.cuda_stream for s in streams}) == 32
    for i, st in enumerate(streams):
        with torch.cuda.stream(st):
            got = sampler._sample_seeded(seeds, fan_out, False, ls)
            for tg, te in zip(got, exp):
                for u, v in zip(tg, te):
                    assert torch.equal(u, v)
        del got
        torch.cuda.synchronize()
        if i == 0:
            torch.cuda.empty_cache()
            per_ctx = free0 - torch.cuda.mem_get_info()[0]
        assert sampler._num_contexts() <= 8
    torch.cuda.empty_cache()
    grown = free0 - torch.cuda.mem_get_info()[0]
    assert per_ctx > 0 and grown <= 10 * per_ctx, (grown, per_ctx)
