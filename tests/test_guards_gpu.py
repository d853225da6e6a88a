"""Range guards and lifetime rules of the library (round 5).

- Every gather (feature server, index_select, the loader's fused label rows) checks each id
  against its source's row count: an id outside [0, rows) -- which the reference reads out of
  bounds (feature_ops.cu:38-73, 140-171), a GPU fault when it is far off -- fills its row from
  row 0 and is reported through the library's async error words; the next gather entry point
  (or dgs.ops._check_async_errors) raises, naming the id.
- Cache lists with an id outside the graph are refused by the constructors.
- PrefetchLoader's batch streams are the library's own, never one of torch's pooled streams
  (which torch hands to every caller round robin), so a batch stream is never the caller's.
- Handles: a pending call whose sampler is gone raises; a wait handle without a wait flag is
  refused (round-3 callers relied on the handle alone).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


def _drain_errors(dgs):
    torch.cuda.synchronize()
    try:
        dgs.ops._check_async_errors()
    except RuntimeError:
        pass


def _small_graph(n=500, seed=1):
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, 30, n)
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, n, int(indptr[-1])).astype(np.int64)
    return torch.from_numpy(indptr), torch.from_numpy(indices)


@pytest.mark.parametrize("cache", ["all", "half"])
def test_feature_gather_out_of_range_id_is_reported(dgs, cache):
    """Strided (whole graph cached) and address-table (partial cache) layouts."""
    n, d = 300, 7
    feats = torch.arange(n * d, dtype=torch.float32).reshape(n, d)
    cn = torch.arange(n) if cache == "all" else torch.arange(0, n, 2)
    srv = dgs.classes.P2PCacheFeatureServer(feats, cn, 0)
    assert srv._layout() == (0 if cache == "all" else -1)
    _drain_errors(dgs)
    nids = torch.tensor([5, n + 3, 17, -1, n - 1], dtype=torch.int64, device="cuda")
    out = srv._CAPI_get_feature(nids)
    torch.cuda.synchronize()
    good = torch.tensor([0, 2, 4])
    assert torch.equal(out.cpu()[good], feats[nids.cpu()[good]])
    # the bad rows are filled from row 0, not read out of bounds
    assert torch.equal(out.cpu()[1], feats[0]) and torch.equal(out.cpu()[3], feats[0])
    # the next gather raises, naming an offending id; then the report is cleared
    with pytest.raises(RuntimeError, match=f"outside \\[0, {n}\\)"):
        srv._CAPI_get_feature(nids[:1])
    dgs.ops._check_async_errors()
    ok = srv._CAPI_get_feature(nids[[0, 2, 4]])
    torch.cuda.synchronize()
    dgs.ops._check_async_errors()
    assert torch.equal(ok.cpu(), feats[nids.cpu()[[0, 2, 4]]])


@pytest.mark.parametrize("nid_dtype", [torch.int64, torch.int32])
def test_index_select_out_of_range_id_is_reported(dgs, nid_dtype):
    data = torch.arange(40, dtype=torch.int64, device="cuda").reshape(20, 2)
    _drain_errors(dgs)
    nids = torch.tensor([3, 20, 19, -7], dtype=nid_dtype, device="cuda")
    out = dgs.ops._CAPI_cuda_index_select(data, nids)
    torch.cuda.synchronize()
    assert torch.equal(out[0], data[3]) and torch.equal(out[2], data[19])
    assert torch.equal(out[1], data[0]) and torch.equal(out[3], data[0])
    with pytest.raises(RuntimeError, match="index_select .* outside \\[0, 20\\)"):
        dgs.ops._check_async_errors()
    dgs.ops._check_async_errors()  # cleared


def test_loader_label_rows_out_of_range_are_reported(dgs):
    """The label gather fused into the feature gather's launch: seeds beyond the label array."""
    from DistGNN.dataloading import PrefetchLoader
    ip, ix = _small_graph()
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    feats = torch.randn(n, 8)
    srv = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(n), 0)
    labels = torch.arange(100, dtype=torch.int64, device="cuda") * 3  # rows 0..99 only
    _drain_errors(dgs)
    seeds = [torch.tensor([1, 2, 3], device="cuda"), torch.tensor([4, 250, 6], device="cuda")]
    got = []
    # the bad seed is in the last batch: the loader itself raises when it is exhausted, naming
    # the batch (no explicit check by the caller)
    with pytest.raises(RuntimeError, match="label gather .* outside \\[0, 100\\).*batch 1\\]"):
        for blocks, x, y in PrefetchLoader(sampler, seeds, [5], server=srv, labels=labels,
                                           depth=2):
            got.append(y.cpu())
    assert got[0].tolist() == [3, 6, 9]
    assert got[1].tolist() == [12, 0, 18]
    dgs.ops._check_async_errors()  # reported once


def test_loader_names_the_batch_of_a_bad_id_and_closes(dgs):
    """A bad id in batch 0 of four is raised by the loader at a later batch's gather entry point
    -- naming batch 0 -- and the loader has closed (its streams are back in the pool)."""
    from DistGNN.dataloading import PrefetchLoader
    from DistGNN.dataloading import prefetch as P
    ip, ix = _small_graph()
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    srv = dgs.classes.P2PCacheFeatureServer(torch.randn(n, 8), torch.arange(n), 0)
    labels = torch.arange(100, dtype=torch.int64, device="cuda")
    _drain_errors(dgs)
    seeds = [torch.tensor([1, 250, 3], device="cuda")] + \
        [torch.tensor([4, 5, 6], device="cuda")] * 3
    loader = PrefetchLoader(sampler, seeds, [5], server=srv, labels=labels, depth=2)
    mine = list(loader._streams)
    handed = 0
    with pytest.raises(RuntimeError, match="outside \\[0, 100\\).*batch 0\\]"):
        for _ in loader:
            handed += 1
            torch.cuda.synchronize()  # batch 0's report is in before the next gather entry
    assert handed == 1
    assert loader._streams == [] and not loader._inflight
    pool = P._FREE_STREAMS.get(torch.device("cuda", 0), [])
    assert len(mine) == 2 and all(any(s is t for t in pool) for s in mine)


def test_cache_lists_outside_the_graph_are_refused(dgs):
    ip, ix = _small_graph()
    n = ip.numel() - 1
    with pytest.raises(RuntimeError, match="cache_nids: an id is outside"):
        dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.tensor([0, 5, n]), 0)
    with pytest.raises(RuntimeError, match="cache_nids: an id is outside"):
        dgs.classes.P2PCacheFeatureServer(torch.randn(n, 4), torch.tensor([-1, 3]), 0)
    # and a valid one still works afterwards
    s = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.tensor([0, 5, n - 1]), 0)
    blocks = s._CAPI_sample_node_classifiction(torch.tensor([0, 5], device="cuda"), [3], False)
    assert int(blocks[0][1].max()) < n


def test_loader_streams_never_alias_pool_streams(dgs):
    """The loader under `with torch.cuda.stream(s)` for each of torch's 32 pooled streams: its
    batch streams are never s (nor any pooled stream), and every batch is bit-exact against
    the sequential loop with the same launch seeds."""
    from DistGNN.dataloading import PrefetchLoader
    ip, ix = _small_graph(2000, seed=3)
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    srv = dgs.classes.P2PCacheFeatureServer(torch.randn(n, 16), torch.arange(n), 0)
    labels = torch.arange(n, device="cuda")
    g = torch.Generator().manual_seed(5)
    batches = [torch.randint(0, n, (64,), generator=g).cuda() for _ in range(4)]
    fan_out = [10, 5]
    dgs.ops._CAPI_set_random_seed(99)
    exp = []
    for s in batches:
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        exp.append((blocks, srv._CAPI_get_feature(blocks[-1][1]), labels[s]))
    torch.cuda.synchronize()
    pool = [torch.cuda.Stream() for _ in range(32)]
    pool_raw = {p.cuda_stream for p in pool}
    assert len(pool_raw) == 32
    for p in pool:
        with torch.cuda.stream(p):
            dgs.ops._CAPI_set_random_seed(99)
            ld = PrefetchLoader(sampler, batches, fan_out, server=srv, labels=labels, depth=3)
            mine = {st.cuda_stream for st in ld._streams}
            assert not mine & pool_raw
            got = list(ld)
            p.synchronize()
        for (gb, gx, gy), (eb, ex, ey) in zip(got, exp):
            for tg, te in zip(gb, eb):
                for u, v in zip(tg, te):
                    assert torch.equal(u, v)
            assert torch.equal(gx, ex) and torch.equal(gy, ey)


def test_wait_handle_without_flag_is_refused(dgs):
    from dgs._lib import lib
    ip, ix = _small_graph()
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    seeds = torch.tensor([1, 2, 3], device="cuda")
    s, L, fo, caps, total, buf, _ = sampler._prepare(seeds, [4, 4], packed=True)
    ev = torch.cuda.Event()
    ev.record()
    st = torch.cuda.current_stream().cuda_stream
    rc = lib.dgs_sampler_sample_begin_after(sampler._h, ctypes.c_void_p(ev.cuda_event),
                                            s.data_ptr(), s.numel(), fo, L, 0, buf.data_ptr(),
                                            None, 0, ctypes.c_void_p(st))
    assert rc != 0
    assert b"without DGS_SAMPLE_WAIT" in lib.dgs_last_error()
    # nothing was begun: a normal call on the stream works
    blocks = sampler._CAPI_sample_node_classifiction(seeds, [4, 4], False)
    assert len(blocks) == 2


def test_pending_call_of_a_destroyed_sampler_raises(dgs):
    ip, ix = _small_graph()
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    p = sampler._sample_begin(torch.tensor([1, 2], device="cuda"), [3, 3], False,
                              host_async=True)
    sampler.__del__()  # what a GC cycle may do before the pending call is ended
    with pytest.raises(RuntimeError, match="destroyed"):
        p.result()
    from dgs._lib import lib
    assert lib.dgs_sampler_sample_end(None, 2, None, None) != 0
    assert lib.dgs_feature_server_destroy(None) == 0


def test_services_never_register_pageable_memory(dgs):
    """Round 6: a sampler / feature server over pageable host arrays never
    registers them.  Fully cached, the arrays only feed the cache build (a device temporary,
    gone when the constructor returns); partly cached, the service reads its host rows from a
    library-owned pinned mirror that goes with it.  Both stay exact against the oracle, the
    caller's tensors stay pageable, and the library holds no registration throughout."""
    import gc
    from oracle import oracle as O
    ip, ix = _small_graph(2000, seed=3)
    n = ip.numel() - 1
    base = dgs.ops._host_memory_state()  # (pins of earlier tests may live on)
    seeds = np.random.default_rng(4).permutation(n)[:300]
    ls = [101, 202, 303]
    exp = O.node_classification_sample(seeds, ip.numpy(), ix.numpy(), [15, 10, 5], False, ls)
    for cache, mirrors in ((torch.arange(n), 0), (torch.arange(0, n, 2), 1)):
        s = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), cache, 0)
        st = dgs.ops._host_memory_state()
        assert st["registrations"] == base["registrations"]
        assert st["mirrors"] == base["mirrors"] + mirrors
        assert not ix.is_pinned() and not ip.is_pinned()
        got = s._sample_seeded(torch.from_numpy(seeds).cuda(), [15, 10, 5], False, ls)
        for g, e in zip(got, exp):
            for a, b in zip(g[1:], e[1:]):
                assert np.array_equal(a.cpu().numpy(), b)
        del s, got
        gc.collect()
        assert dgs.ops._host_memory_state() == base
    rng = np.random.default_rng(5)
    data = torch.from_numpy(rng.standard_normal((n, 24)).astype(np.float32))
    q = rng.integers(0, n, 4096)
    for cache, mirrors in ((torch.arange(n), 0), (torch.arange(1, n, 3), 1)):
        fs = dgs.classes.P2PCacheFeatureServer(data, cache, 0)
        st = dgs.ops._host_memory_state()
        assert st["registrations"] == base["registrations"]
        assert st["mirrors"] == base["mirrors"] + mirrors
        assert not data.is_pinned()
        assert np.array_equal(fs._CAPI_get_feature(torch.from_numpy(q).cuda()).cpu().numpy(),
                              O.index_select(data.numpy(), q))
        del fs
        gc.collect()
        assert dgs.ops._host_memory_state() == base


def test_empty_seed_batch(dgs):
    """A batch of no seeds (a train split's empty tail): every hop's frontier and COO are empty,
    synchronously and through the loader, and the calls around it stay exact.  (Round 6: the
    compaction published no sizes for an empty call -- 'sizes were not published'.)"""
    from DistGNN.dataloading import PrefetchLoader
    from oracle import oracle as O
    ip, ix = _small_graph(800, seed=9)
    n = ip.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(), torch.arange(n), 0)
    empty = torch.empty(0, dtype=torch.int64, device="cuda")
    for replace in (False, True):
        blocks = sampler._CAPI_sample_node_classifiction(empty, [5, 4, 3], replace)
        assert len(blocks) == 3
        for _, f, r, c in blocks:
            assert f.numel() == 0 and r.numel() == 0 and c.numel() == 0
    seeds = [torch.tensor([3, 9, 27], device="cuda"), empty, torch.tensor([5, 1], device="cuda")]
    dgs.ops._CAPI_set_random_seed(31)
    ls = dgs.ops.draw_launch_seeds(9)
    dgs.ops._CAPI_set_random_seed(31)
    got = [b for b, _, _ in PrefetchLoader(sampler, seeds, [5, 4, 3], depth=3)]
    for i, (s, b) in enumerate(zip(seeds, got)):
        exp = O.node_classification_sample(s.cpu().numpy(), ip.numpy(), ix.numpy(), [5, 4, 3],
                                           False, ls[3 * i:3 * i + 3]) if s.numel() else None
        for h, (_, f, r, c) in enumerate(b):
            if exp is None:
                assert f.numel() == r.numel() == c.numel() == 0
            else:
                assert np.array_equal(f.cpu().numpy(), exp[h][1])
                assert np.array_equal(c.cpu().numpy(), exp[h][3])
