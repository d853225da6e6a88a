"""GPU parity: the HIP path (libdgs_amd.so through the `dgs` binding) against the CPU oracle.

Bar: bit-exact for sampled indices, frontiers, relabeled COO and every gather (a byte copy);
the heat ops use float atomics in the reference, so they are compared with rtol 1e-5.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def dgs():
    import dgs as _dgs
    return _dgs


def _gold():
    return np.load(os.path.join(GOLD, "sampler_golden.npz"))


def _hub_graph(seed=0, giant=True):
    """Small graph with degree-0 rows, deg == k rows and hub rows (deg >> 1024 + k).
    giant=False drops the 250K-degree row (float-atomic heat sums over it are order
    dependent beyond the 1e-5 tolerance, preprocess_heat.cu uses atomicAdd too)."""
    rng = np.random.default_rng(seed)
    n = 400
    degs = rng.integers(0, 80, n)
    degs[:6] = [0, 1, 5, 15, 3000, 9000]
    degs[6:10] = [130, 512, 1040, 1100]
    degs[10:12] = [2600, 250000 if giant else 2700]  # hub chunks on both modulo paths
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, n, int(indptr[-1])).astype(np.int64)
    probs = (rng.random(indices.size) + 0.01).astype(np.float32)
    probs[::13] = 0.0
    return indptr, indices, probs


def _cuda(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


# ------------------------------------------------------------------ gather
@pytest.mark.parametrize("dim", [1, 3, 100, 128, 256, 257])
@pytest.mark.parametrize("nid_dtype", [torch.int64, torch.int32])
def test_index_select_matches_oracle(dgs, dim, nid_dtype):
    rng = np.random.default_rng(dim)
    data = rng.standard_normal((5000, dim)).astype(np.float32)
    nids = rng.integers(0, 5000, 7777)
    got = dgs.ops._CAPI_cuda_index_select(_cuda(data), _cuda(nids, nid_dtype))
    exp = O.index_select(data, nids)
    assert got.shape == (7777, dim)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), exp.view(np.uint32))


def test_index_select_labels_pinned_host(dgs):
    labels = torch.arange(1000, dtype=torch.int64) * 7
    labels = labels.pin_memory()
    nids = torch.randint(0, 1000, (333,), device="cuda")
    got = dgs.ops._CAPI_cuda_index_select(labels, nids)
    assert got.is_cuda and torch.equal(got.cpu(), labels[nids.cpu()])
    lab3 = torch.arange(3000, dtype=torch.float32).reshape(1000, 3)
    dgs.ops._CAPI_tensor_pin_memory(lab3)
    got = dgs.ops._CAPI_cuda_index_select(lab3, nids)
    assert torch.equal(got.cpu(), lab3[nids.cpu()])
    dgs.ops._CAPI_tensor_unpin_memory(lab3)


def test_index_select_empty(dgs):
    data = torch.randn(10, 4, device="cuda")
    out = dgs.ops._CAPI_cuda_index_select(data, torch.empty(0, dtype=torch.int64, device="cuda"))
    assert out.shape == (0, 4)


# ------------------------------------------------------------------ standalone sampling
@pytest.mark.parametrize("k", [1, 5, 15, 40, 130])
@pytest.mark.parametrize("replace", [False, True])
def test_sample_neighbors_uniform(dgs, k, replace):
    indptr, indices, _ = _hub_graph(k)
    seeds = np.random.default_rng(k).permutation(indptr.size - 1)[:300]
    seeds = np.concatenate([np.arange(10), seeds])
    for s in (1, 2):
        dgs.ops._CAPI_set_random_seed(1000 * k + s)
        ls = O.launch_seeds(1000 * k + s, 1)[0]
        row, col = dgs.ops._CAPI_cuda_sample_neighbors(_cuda(seeds), _cuda(indptr),
                                                       _cuda(indices), k, replace)
        er, ec = O.sample_uniform(seeds, indptr, indices, k, replace, ls)
        assert np.array_equal(row.cpu().numpy(), er)
        assert np.array_equal(col.cpu().numpy(), ec)


@pytest.mark.parametrize("k", [1, 4, 15, 32])
@pytest.mark.parametrize("replace", [False, True])
def test_sample_neighbors_bias(dgs, k, replace):
    indptr, indices, probs = _hub_graph(7 + k)
    seeds = np.concatenate([np.arange(10), np.random.default_rng(k).integers(0, 400, 200)])
    dgs.ops._CAPI_set_random_seed(77 + k)
    ls = O.launch_seeds(77 + k, 1)[0]
    row, col = dgs.ops._CAPI_cuda_sample_neighbors_bias(_cuda(seeds), _cuda(indptr),
                                                        _cuda(indices), _cuda(probs), k, replace)
    er, ec = O.sample_bias(seeds, indptr, indices, probs, k, replace, ls)
    assert np.array_equal(row.cpu().numpy(), er)
    assert np.array_equal(col.cpu().numpy(), ec)


def _bias_hub_graph(seed):
    """Biased hub rows of every class of the streaming scheme (csrc/sample.hip): rows the boot
    kernel's sample covers whole (deg <= 4096) and larger ones up to 250K edges, a row with
    all-zero weights (no finite sample threshold) and one with only three positive weights,
    rows with infinite weights (tied keys), plus ordinary rows."""
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, 60, 300)
    # (round 5: rows of 3800 / 4000 edges have exactly the 16 chunks the boot draws -- nothing
    # left for the stream -- and 4020 / 4300 leave one / two chunks to it)
    hubs = [2049, 3000, 5000, 8192, 8193, 9000, 20000, 30000, 70000, 250000, 3800, 4000, 4020,
            4300]
    degs[:len(hubs)] = hubs
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, degs.size, int(indptr[-1])).astype(np.int64)
    probs = (rng.random(indices.size) + 0.01).astype(np.float32)
    probs[::17] = 0.0
    probs[indptr[6]:indptr[7]] = 0.0             # deg 20000: all zero
    probs[indptr[7]:indptr[8]] = 0.0             # deg 30000: three positive weights
    probs[indptr[7] + np.array([5, 17000, 29999])] = [0.5, 2.0, 1.0]
    # deg 70000: weights rising along the row (a prefix sample would be unrepresentative)
    probs[indptr[8]:indptr[9]] = np.linspace(0.01, 50.0, 70000, dtype=np.float32)
    # infinite weights (keys +-0, tied: picked by edge index): 40 in a streamed row, 20 in a row
    # the boot covers whole, 3 in a small row
    probs[indptr[5] + rng.choice(9000, 40, replace=False)] = np.inf
    probs[indptr[2] + rng.choice(5000, 20, replace=False)] = np.inf
    small = int(np.argmax(degs[10:] >= 40)) + 10
    probs[indptr[small] + np.array([0, 7, 30])] = np.inf
    return indptr, indices, probs


@pytest.mark.parametrize("cap", [None, "0", "40"])
@pytest.mark.parametrize("k", [1, 5, 15, 32])
def test_bias_hub_rows_streaming(dgs, k, cap, monkeypatch):
    """Every class of biased hub row bit-exact against the oracle; DGS_BIAS_TEST_CAP squeezes the
    streamed rows' candidate lists so they overflow and are recomputed exactly."""
    if cap is not None:
        monkeypatch.setenv("DGS_BIAS_TEST_CAP", cap)
    indptr, indices, probs = _bias_hub_graph(3 + k)
    n = indptr.size - 1
    rng = np.random.default_rng(k)
    seeds = np.concatenate([np.arange(10), rng.integers(0, n, 150), np.arange(10)])  # repeats
    for s in (1, 2):
        dgs.ops._CAPI_set_random_seed(900 + 10 * k + s)
        ls = O.launch_seeds(900 + 10 * k + s, 1)[0]
        row, col = dgs.ops._CAPI_cuda_sample_neighbors_bias(_cuda(seeds), _cuda(indptr),
                                                            _cuda(indices), _cuda(probs), k,
                                                            False)
        er, ec = O.sample_bias(seeds, indptr, indices, probs, k, False, ls)
        assert np.array_equal(row.cpu().numpy(), er)
        assert np.array_equal(col.cpu().numpy(), ec)


def test_bias_filter_bounds_are_sound(dgs):
    """The biased kernels' only inequalities: the hub sampling threshold is built from
    key_lower() (it must never exceed the exact key), and edges are dropped by two cheap tests
    (they must only fire when the exact key is strictly below the threshold, ties included).
    4 M random draws with log-uniform and integer (degree-like) weights plus edge values of both
    (0, -1, denormals, the key_lower range limits, 1e38, inf, NaN; draws at 0 and near 2^32),
    each against thresholds at and around its own exact key, which must also match the oracle
    bit for bit."""
    rng = np.random.default_rng(31)
    n = 1 << 22
    x = rng.integers(0, 2 ** 32, n, dtype=np.uint64)
    ex = np.array([0, 1, 2, 255, 256, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 1, 2 ** 32 - 2, 2 ** 32 - 128,
                   2 ** 32 - 129, 2 ** 32 - 256, 2 ** 32 - 512, 2 ** 32 - 4608, 2 ** 32 - 4609,
                   2 ** 32 - 8192], dtype=np.uint64)
    p = np.exp(rng.uniform(np.log(1e-6), np.log(1e6), n)).astype(np.float32)
    p[1::3] = rng.integers(1, 200000, p[1::3].size).astype(np.float32)
    ep = np.array([0.0, -0.0, -1.0, 1e-45, 1e-40, 7.8e-31, 7.888609052210118e-31, 1e-30, 0.5, 1.0,
                   1e30, 1.2676506002282294e30, 1.3e30, 1e38, np.inf, np.nan], dtype=np.float32)
    # every edge draw with every edge weight, repeated at the front
    gx, gp = np.meshgrid(ex, ep)
    m = gx.size
    x[:m], p[:m] = gx.ravel(), gp.ravel()
    x[m:2 * m], p[m:2 * m] = gx.ravel(), rng.uniform(0.5, 3.0, m).astype(np.float32)
    key = O.ares_keys(O.curand_uniform_of(x), p)
    # thresholds at, just above / below and around each key; -inf keys get random thresholds
    fac = np.array([1.0, 1.0 + 2 ** -24, 1.0 - 2 ** -24, 1.0 + 2 ** -20, 1.0 - 2 ** -20,
                    1.0 + 2 ** -16, 1.0 - 2 ** -16, 1.0 + 2 ** -12, 1.0 - 2 ** -12, 1.5, 0.5, 4.0],
                   dtype=np.float32)
    thr = key * fac[rng.integers(0, fac.size, n)]
    ties = rng.random(n) < 0.2
    thr[ties] = key[ties]
    bad = ~np.isfinite(thr)
    thr[bad] = -np.exp(rng.uniform(np.log(1e-9), np.log(1e3), int(bad.sum()))).astype(np.float32)
    thr[:16] = 0.0
    gk, gl, gf = dgs.ops._Test_BiasKeyBounds(_cuda(x.astype(np.int64)), _cuda(p), _cuda(thr))
    gk, gl, gf = gk.cpu().numpy(), gl.cpu().numpy(), gf.cpu().numpy()
    assert np.array_equal(gk.view(np.uint32), key.view(np.uint32)), "exact key differs from oracle"
    assert not np.isnan(gk).any()
    assert (gl <= gk).all(), "key_lower above the exact key"
    for bit, name in ((1, "streamed-hub filter"), (2, "row filter")):
        fired = (gf & bit) != 0
        assert (gk[fired] < thr[fired]).all(), f"{name} dropped an edge whose key reaches thr"
        assert fired.mean() > 0.05, f"{name} never fires (test inputs too weak)"


def test_sample_golden_vectors(dgs):
    z = _gold()
    seeds, indptr, indices, probs = z["seeds"], z["indptr"], z["indices"], z["probs"]
    # the fixture's launch seeds are mt19937_64(7) outputs 0..15
    i = 0
    for k in (3, 5, 15, 40):
        for rep in (0, 1):
            dgs.ops._CAPI_set_random_seed(7)
            for _ in range(i % 16):
                dgs.ops._Test_Randn()
            r, c = dgs.ops._CAPI_cuda_sample_neighbors(_cuda(seeds), _cuda(indptr),
                                                       _cuda(indices), k, bool(rep))
            assert np.array_equal(r.cpu().numpy(), z[f"uniform_k{k}_r{rep}_row"])
            assert np.array_equal(c.cpu().numpy(), z[f"uniform_k{k}_r{rep}_col"])
            if k <= 32:
                dgs.ops._CAPI_set_random_seed(7)
                for _ in range(i % 16):
                    dgs.ops._Test_Randn()
                r, c = dgs.ops._CAPI_cuda_sample_neighbors_bias(
                    _cuda(seeds), _cuda(indptr), _cuda(indices), _cuda(probs), k, bool(rep))
                assert np.array_equal(r.cpu().numpy(), z[f"bias_k{k}_r{rep}_row"])
                assert np.array_equal(c.cpu().numpy(), z[f"bias_k{k}_r{rep}_col"])
            i += 1


def test_sample_empty_and_zero_picks(dgs):
    indptr, indices, _ = _hub_graph()
    e = torch.empty(0, dtype=torch.int64, device="cuda")
    r, c = dgs.ops._CAPI_cuda_sample_neighbors(e, _cuda(indptr), _cuda(indices), 5, False)
    assert r.numel() == 0 and c.numel() == 0
    s = _cuda(np.arange(20))
    r, c = dgs.ops._CAPI_cuda_sample_neighbors(s, _cuda(indptr), _cuda(indices), 0, False)
    assert r.numel() == 0


# ------------------------------------------------------------------ relabel
def test_relabel_matches_oracle(dgs):
    rng = np.random.default_rng(3)
    for n in (0, 1, 17, 5000):
        a = rng.integers(0, 300, n)
        b = rng.integers(0, 600, 3 * n)
        uniq, (ra, rb) = dgs.ops._CAPI_cuda_sampled_tensor_relabel([_cuda(a), _cuda(b)],
                                                                  [_cuda(a), _cuda(b)])
        eu, (ea, eb) = O.relabel([a, b], [a, b])
        assert np.array_equal(uniq.cpu().numpy(), eu)
        assert np.array_equal(ra.cpu().numpy(), ea) and np.array_equal(rb.cpu().numpy(), eb)
    uniq, (r,) = dgs.ops._CAPI_cuda_sampled_tensor_relabel([_cuda([5, 6])], [_cuda([6, 7, 5])])
    assert uniq.tolist() == [5, 6] and r.tolist() == [1, -1, 0]


# ------------------------------------------------------------------ extract / KATs
def test_reference_extract_kat(dgs):
    with open(os.path.join(GOLD, "reference_kats.json")) as f:
        k = json.load(f)
    g, e = k["toy_graph"], k["extract"]
    indptr = torch.tensor(g["indptr"]).cuda()
    nids = torch.tensor(e["cache_nids"]).cuda()
    sub = dgs.ops._Test_ExtractIndptr(nids, indptr)
    assert sub.tolist() == e["sub_indptr"]
    assert dgs.ops._Test_ExtractEdgeData(nids, indptr, sub,
                                         torch.tensor(g["indices"]).cuda()).tolist() == \
        e["sub_indices"]
    probs = torch.tensor(g["probs"], dtype=torch.float32).cuda()
    assert torch.equal(dgs.ops._Test_ExtractEdgeData(nids, indptr, sub, probs).cpu(),
                       torch.tensor(e["sub_probs"], dtype=torch.float32))
    for nids_r, exp in zip(k["p2p_server"]["rank_cache_nids"], k["p2p_server"]["rank_sub_indptr"]):
        assert dgs.ops._Test_ExtractIndptr(torch.tensor(nids_r).cuda(), indptr).tolist() == exp


def test_reference_feature_server_kat(dgs):
    with open(os.path.join(GOLD, "reference_kats.json")) as f:
        k = json.load(f)["feature_server"]
    feat = torch.arange(0, 100, 1).float().pin_memory().reshape(10, 10)
    fs = dgs.classes.P2PCacheFeatureServer(feat, torch.tensor(k["rank_cache_nids"][0]).cuda(), 0)
    got = fs._CAPI_get_feature(torch.tensor(k["query"]).cuda())
    assert got.tolist() == [[float(x) for x in row] for row in k["expected"]]
    assert torch.equal(fs._CAPI_get_cpu_feature(), feat)
    assert torch.equal(fs._CAPI_get_gpu_feature().cpu(), feat[[0, 3]])


# ------------------------------------------------------------------ services
@pytest.mark.parametrize("cache", ["all", "half", "none_but_one"])
@pytest.mark.parametrize("replace", [False, True])
@pytest.mark.parametrize("bias", [False, True])
def test_p2p_cache_sampler_matches_oracle(dgs, cache, replace, bias):
    indptr, indices, probs = _hub_graph(11)
    n = indptr.size - 1
    if cache == "all":
        cnids = np.random.default_rng(0).permutation(n)
    elif cache == "half":
        cnids = np.random.default_rng(1).permutation(n)[: n // 2]
    else:
        cnids = np.array([3])
    pr = torch.from_numpy(probs) if bias else torch.Tensor()
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices), pr,
                                          torch.from_numpy(cnids), 0)
    seeds = np.random.default_rng(5).permutation(n)[:64]
    seeds[:6] = np.arange(6)
    fan_out = [15, 10, 5] if not bias else [8, 5, 3]
    dgs.ops._CAPI_set_random_seed(4242)
    got = sampler._CAPI_sample_node_classifiction(_cuda(seeds), fan_out, replace)
    exp = O.node_classification_sample(seeds, indptr, indices, fan_out, replace,
                                       O.launch_seeds(4242, 3), probs=probs if bias else None)
    assert len(got) == len(exp) == 3
    for (gs, gf, gr, gc), (es, ef, er, ec) in zip(got, exp):
        assert np.array_equal(gs.cpu().numpy(), es)
        assert np.array_equal(gf.cpu().numpy(), ef)
        assert np.array_equal(gr.cpu().numpy(), er)
        assert np.array_equal(gc.cpu().numpy(), ec)


@pytest.mark.parametrize("bad", [-1, "n", 1 << 40])
def test_sampler_rejects_out_of_range_seed(dgs, bad):
    # The reference reads out of bounds here; this path samples the bad row as empty, keeps it
    # out of the relabel table and raises after the call.  The tables must stay clean: the next
    # call is still bit-exact.
    indptr, indices, probs = _hub_graph(11)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(0, n, 2), 0)
    seeds = np.random.default_rng(5).permutation(n)[:64]
    badseeds = seeds.copy()
    badseeds[7] = n if bad == "n" else bad
    with pytest.raises(RuntimeError, match="outside"):
        sampler._CAPI_sample_node_classifiction(_cuda(badseeds), [15, 10, 5], False)
    dgs.ops._CAPI_set_random_seed(99)
    got = sampler._CAPI_sample_node_classifiction(_cuda(seeds), [15, 10, 5], False)
    exp = O.node_classification_sample(seeds, indptr, indices, [15, 10, 5], False,
                                       O.launch_seeds(99, 3))
    for g, e in zip(got, exp):
        for a, b in zip(g, e):
            assert np.array_equal(a.cpu().numpy(), b)


def test_sampler_getters(dgs):
    with open(os.path.join(GOLD, "reference_kats.json")) as f:
        g = json.load(f)["toy_graph"]
    indptr = torch.tensor(g["indptr"]).pin_memory()
    indices = torch.tensor(g["indices"]).pin_memory()
    probs = torch.tensor(g["probs"]).pin_memory()
    s = dgs.classes.P2PCacheSampler(indptr, indices, probs, torch.tensor([0, 3]), 0)
    ip, ix, pr = s._CAPI_get_cpu_structure_tensors()
    assert ip is indptr and ix is indices and pr is probs
    si, sx, sp = s._CAPI_get_local_cache_structure_tensors()
    assert si.tolist() == [0, 4, 4] and sx.tolist() == [1, 2, 3, 4]
    assert torch.allclose(sp.cpu(), torch.tensor([0.1, 0.2, 0.3, 0.4]))
    key, idx, devid = s._local_cache_map_compact()
    assert key.tolist() == [0, 3] and idx.tolist() == [0, 1] and devid.tolist() == [0, 0]
    # the reference's own layout (hashmap.cu:15-77): 2 * _UpPower(2) = 8 slots; two keys on
    # distinct home slots land there, so it equals the sequential restatement slot for slot
    key, idx, devid = s._CAPI_get_local_cache_hashmap_tensors()
    ek, ei, ed = O.cache_hashmap([np.array([0, 3])], 0)
    assert key.dtype == torch.int64 and len(key) == 8
    assert key.tolist() == ek.tolist() and idx.tolist() == ei.tolist()
    assert devid.tolist() == ed.tolist()
    # reference test_sampler_bias.py: seeds [0, 3, 5], fan-out [2, 2]
    res = s._CAPI_sample_node_classifiction(torch.tensor([0, 3, 5]).cuda(), [2, 2], False)
    assert res[0][1][:3].tolist() == [0, 3, 5]


@pytest.mark.parametrize("id_dtype", [torch.int64, torch.int32])
def test_reference_cache_hashmap(dgs, id_dtype):
    """_CAPI_get_local_cache_hashmap_tensors returns the reference's open-addressing map
    (hashmap.cu:15-77) in the cache list's id type: capacity 2 * _UpPower(n), key set, -1 where
    empty, and every cached node's (idx, devid) reached by the reference's probe sequence;
    a list with no colliding home slots lands slot for slot where the restatement puts it."""
    rng = np.random.default_rng(12)
    n = 20000
    ip = torch.from_numpy(np.arange(0, 2 * n + 1, 2, dtype=np.int64))
    ix = torch.from_numpy(rng.integers(0, n, 2 * n).astype(np.int64))
    ib = 8 if id_dtype == torch.int64 else 4
    for cache in (rng.choice(n, 5000, replace=False), np.array([17, 4, 9999])):
        s = dgs.classes.P2PCacheSampler(ip, ix, torch.Tensor(),
                                        torch.from_numpy(cache).to(id_dtype), 0)
        key, idx, devid = s._CAPI_get_local_cache_hashmap_tensors()
        assert key.dtype == id_dtype and idx.dtype == id_dtype
        key, idx, devid = (t.cpu().numpy().astype(np.int64) for t in (key, idx, devid))
        assert len(key) == O.cache_hashmap_dir_size(cache.size)
        assert sorted(key[key >= 0].tolist()) == sorted(cache.tolist())
        assert (idx[key < 0] == -1).all() and (devid[key < 0] == -1).all()
        for i, v in enumerate(cache.tolist()):
            pos = O.cache_hashmap_find(key, v, ib)
            assert pos >= 0 and idx[pos] == i and devid[pos] == 0
        ek, ei, ed = O.cache_hashmap([cache], 0, ib)
        homes = [O._home(int(v), len(ek), ib) for v in cache.tolist()]
        if len(set(homes)) == len(homes):
            assert key.tolist() == ek.tolist() and idx.tolist() == ei.tolist()


def test_feature_server_matches_oracle(dgs):
    rng = np.random.default_rng(9)
    data = rng.standard_normal((3000, 100)).astype(np.float32)
    for cnids, layout in ((np.arange(3000), 0), (rng.permutation(3000)[:1000], -1),
                          (np.array([7]), -1), (rng.permutation(3000), -1)):
        fs = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(data), torch.from_numpy(cnids), 0)
        assert fs._layout() == layout  # identity layout -> computed addresses, no table
        q = rng.integers(0, 3000, 4096)
        got = fs._CAPI_get_feature(_cuda(q))
        assert np.array_equal(got.cpu().numpy(), O.index_select(data, q))


@pytest.mark.parametrize("dim,dtype", [(33, np.float32), (1, np.int64), (3, np.int16),
                                       (128, np.float32), (7, np.uint8)])
def test_feature_server_row_sizes(dgs, dim, dtype):
    """Every vector width of the gather (16/8/4/2/1-byte chunks), both address layouts."""
    rng = np.random.default_rng(dim)
    data = (rng.standard_normal((777, dim)) * 100).astype(dtype)
    for cnids in (np.arange(777), rng.permutation(777)[:300]):
        fs = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(data), torch.from_numpy(cnids), 0)
        q = np.concatenate([rng.integers(0, 777, 999), [0, 776]])
        got = fs._CAPI_get_feature(_cuda(q)).cpu().numpy()
        assert np.array_equal(got, data[q])


def test_tensor_p2p_server_local(dgs):
    t = torch.arange(12, dtype=torch.int64, device="cuda").reshape(4, 3)
    srv = dgs.classes.TensorP2PServer(t)
    assert torch.equal(srv._CAPI_get_local_device_tensor(), t)
    assert torch.equal(srv._CAPI_get_device_tensor(0), t.flatten())


@pytest.mark.parametrize("n_seeds,fan_out,replace", [(1 << 20, [2048], True),
                                                      (1 << 22, [512], False),
                                                      (1 << 23, [300], True)])
def test_sampler_rejects_int32_position_overflow(dgs, n_seeds, fan_out, replace):
    """Relabel positions are 32-bit: a call whose hop could hold 2^31 - 1 or more seeds +
    sampled edges (host-side bounds) raises before anything is allocated or launched, and the
    sampler stays usable."""
    indptr, indices, _ = _hub_graph(11)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(n), 0)
    seeds = torch.zeros(n_seeds, dtype=torch.int64, device="cuda")
    with pytest.raises(RuntimeError, match="32-bit"):
        sampler._CAPI_sample_node_classifiction(seeds, fan_out, replace)
    small = _cuda(np.random.default_rng(5).permutation(n)[:64])
    dgs.ops._CAPI_set_random_seed(99)
    got = sampler._CAPI_sample_node_classifiction(small, [15, 10, 5], False)
    exp = O.node_classification_sample(small.cpu().numpy(), indptr, indices, [15, 10, 5], False,
                                       O.launch_seeds(99, 3))
    for g, e in zip(got, exp):
        for a, b in zip(g, e):
            assert np.array_equal(a.cpu().numpy(), b)


# ------------------------------------------------------------------ heat
@pytest.mark.parametrize("bias", [False, True])
def test_heat_matches_oracle(dgs, bias):
    indptr, indices, probs = _hub_graph(2, giant=False)
    probs = probs + np.float32(0.05)
    n = indptr.size - 1
    heat = np.random.default_rng(1).random(n).astype(np.float32)
    seeds = np.random.default_rng(2).permutation(n)[:150]
    if bias:
        got = dgs.ops._CAPI_compute_frontier_heat_with_bias(
            _cuda(seeds), _cuda(indptr), _cuda(indices), _cuda(probs), _cuda(heat), 5, 0)
    else:
        got = dgs.ops._CAPI_compute_frontier_heat(_cuda(seeds), _cuda(indptr), _cuda(indices),
                                                  _cuda(heat), 5, 0)
    exp = O.frontier_heat(seeds, indptr, indices, heat, 5, probs=probs if bias else None)
    np.testing.assert_allclose(got.cpu().numpy(), exp, rtol=1e-5, atol=1e-6)


def test_heat_uva_host_graph(dgs):
    indptr, indices, _ = _hub_graph(4, giant=False)
    n = indptr.size - 1
    ip, ix = torch.from_numpy(indptr), torch.from_numpy(indices)
    dgs.ops._CAPI_tensor_pin_memory(ip)
    dgs.ops._CAPI_tensor_pin_memory(ix)
    heat = torch.rand(n, device="cuda")
    seeds = torch.arange(0, n, 3, device="cuda")
    got = dgs.ops._CAPI_compute_frontier_heat(seeds, ip, ix, heat, 10, 0)
    exp = O.frontier_heat(seeds.cpu().numpy(), indptr, indices, heat.cpu().numpy(), 10)
    np.testing.assert_allclose(got.cpu().numpy(), exp, rtol=1e-5, atol=1e-6)
    dgs.ops._CAPI_tensor_unpin_memory(ip)
    dgs.ops._CAPI_tensor_unpin_memory(ix)


# ------------------------------------------------------------------ degree boundaries
def _degree_graph(degs, seed):
    """Rows of exactly the given degrees (random neighbour ids) and random probabilities with
    some zeros."""
    rng = np.random.default_rng(seed)
    degs = np.asarray(degs, dtype=np.int64)
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, degs.size, int(indptr[-1])).astype(np.int64)
    probs = (rng.random(indices.size) + 0.01).astype(np.float32)
    probs[::29] = 0.0
    return indptr, indices, probs


def _uniform_boundary_degrees(k, huge):
    """Every degree class of the uniform sampler (csrc/sample.hip) around its limits: copy
    (deg <= k), row reservoir (deg - k <= kHubT = 128), hub chunks of 512 edges, and the hub
    chunks' modulo forms -- mod_mid below d = 8192 (24-bit product from d = 257), mod_big from
    d = 4096 (24-bit product below 2^24) and the generic % in between."""
    d = [0, 1, k - 1, k, k + 1, k + 127, k + 128, k + 129, k + 130, k + 128 + 512,
         k + 129 + 512, k + 129 + 1024, 256, 257, 258, 768, 769, 4095, 4096, 4097, k + 4096,
         k + 4097, 7680, 7681, 8192, 8193, k + 8192, k + 8193, 8704, 12345, 65537]
    if huge:
        d += [(1 << 24) - 200, (1 << 24) + 700]  # chunks on both sides of 2^24
    return sorted({x for x in d if x >= 0})


@pytest.mark.parametrize("k,replace,huge", [(1, False, False), (5, False, True),
                                            (15, False, False), (100, False, False),
                                            (129, False, False), (15, True, False),
                                            (64, True, True)])
def test_uniform_degree_boundaries(dgs, k, replace, huge):
    """Rows at every degree limit of the uniform sampler, each sampled once and again as a
    repeated seed, bit-exact with the oracle for two launch seeds."""
    indptr, indices, _ = _degree_graph(_uniform_boundary_degrees(k, huge), 17 + k)
    n = indptr.size - 1
    seeds = np.concatenate([np.arange(n), np.arange(n)[::-3]])
    ip, ix = _cuda(indptr), _cuda(indices)
    for s in (1, 2):
        dgs.ops._CAPI_set_random_seed(5000 + 10 * k + s)
        ls = O.launch_seeds(5000 + 10 * k + s, 1)[0]
        row, col = dgs.ops._CAPI_cuda_sample_neighbors(_cuda(seeds), ip, ix, k, replace)
        er, ec = O.sample_uniform(seeds, indptr, indices, k, replace, ls)
        assert np.array_equal(row.cpu().numpy(), er)
        assert np.array_equal(col.cpu().numpy(), ec)


@pytest.mark.parametrize("k,replace", [(1, False), (16, False), (32, False), (8, True)])
def test_bias_degree_boundaries(dgs, k, replace):
    """Rows around the biased sampler's limits: deg <= k, the hub limit (deg > kBiasHubT =
    1024), whole 256-edge stream chunks and one edge past them, the boot sample's 4096 edges,
    and a long row."""
    degs = [0, 1, k - 1, k, k + 1, 33, 64, 65, 1023, 1024, 1025, 1280, 1281, 2047, 2048, 2049,
            4095, 4096, 4097, 4352, 4353, 8191, 8193, 65536, 1 << 20]
    indptr, indices, probs = _degree_graph(sorted({d for d in degs if d >= 0}), 3 + k)
    n = indptr.size - 1
    seeds = np.concatenate([np.arange(n), np.arange(n)[::-2]])
    dgs.ops._CAPI_set_random_seed(7000 + k)
    ls = O.launch_seeds(7000 + k, 1)[0]
    row, col = dgs.ops._CAPI_cuda_sample_neighbors_bias(_cuda(seeds), _cuda(indptr),
                                                        _cuda(indices), _cuda(probs), k, replace)
    er, ec = O.sample_bias(seeds, indptr, indices, probs, k, replace, ls)
    assert np.array_equal(row.cpu().numpy(), er)
    assert np.array_equal(col.cpu().numpy(), ec)


# ------------------------------------------------------------------ larger graph
def test_rmat_scale16_sampler_bit_exact(dgs):
    from DistGNN.dataloading.synthetic import rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(16, 12, seed=20261015)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(n), 0)
    seeds = np.random.default_rng(2).permutation(n)[:1024]
    dgs.ops._CAPI_set_random_seed(99)
    got = sampler._CAPI_sample_node_classifiction(_cuda(seeds), [15, 10, 5], False)
    exp = O.node_classification_sample(seeds, indptr, indices, [15, 10, 5], False,
                                       O.launch_seeds(99, 3))
    for (gs, gf, gr, gc), (es, ef, er, ec) in zip(got, exp):
        assert np.array_equal(gf.cpu().numpy(), ef)
        assert np.array_equal(gr.cpu().numpy(), er)
        assert np.array_equal(gc.cpu().numpy(), ec)


@pytest.mark.parametrize("n_seeds,k,replace,dup", [
    (1365, 5, False, False),   # S + S k = 8190 elements of cat(seeds, col): 8 compaction tiles
    (1366, 5, False, False),   # 8196: a ninth, nearly empty tile
    (2048, 3, False, True),    # exactly 8192, repeated seeds: rows checked and relabelled
    (2048, 3, True, True),
    (1200, 5, True, False),
    (1, 7, False, False),      # one row: one sampling workgroup, one tile
])
def test_first_hop_compaction_tile_boundary(dgs, n_seeds, k, replace, dup):
    """First hops at the tile boundaries of the compaction (k_dcount / k_dscatter, 1024-element
    tiles) and at the 8192-element limit of the rejected fused-compaction variant
    (profiles/r06_ab_fused_compaction_rejected.txt): bit-exact with the oracle, twice in a row
    (the tables' clean-up), and the second hop over the first hop's frontier."""
    from DistGNN.dataloading.synthetic import rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(14, 12, seed=31)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.Tensor(), torch.arange(n), 0)
    rng = np.random.default_rng(n_seeds + k)
    seeds = rng.integers(0, n, n_seeds) if dup else rng.permutation(n)[:n_seeds]
    fan_out = [4, k]
    for rep in range(2):  # the workgroup counter is reset by the launch that used it
        dgs.ops._CAPI_set_random_seed(77 + rep)
        got = sampler._CAPI_sample_node_classifiction(_cuda(seeds), fan_out, replace)
        exp = O.node_classification_sample(seeds, indptr, indices, fan_out, replace,
                                           O.launch_seeds(77 + rep, 2))
        for (gs, gf, gr, gc), (es, ef, er, ec) in zip(got, exp):
            assert np.array_equal(gf.cpu().numpy(), ef)
            assert np.array_equal(gr.cpu().numpy(), er)
            assert np.array_equal(gc.cpu().numpy(), ec)


@pytest.mark.parametrize("fan_out,replace", [([15, 10, 5], False), ([25, 10], False),
                                             ([8, 4, 2], True)])
def test_rmat_biased_multihop_bit_exact(dgs, fan_out, replace):
    """Degree-weighted biased sampling over a power-law graph: hub rows split across
    half-waves (chain RNG offsets, batched top-k merges) and the row kernel, 2-3 hops."""
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_numpy
    indptr, indices = rmat_csc_numpy(14, 16, seed=7)
    probs = degree_probs(indptr, indices)
    n = indptr.size - 1
    sampler = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                          torch.from_numpy(probs), torch.arange(n), 0)
    seeds = np.random.default_rng(5).permutation(n)[:700]
    dgs.ops._CAPI_set_random_seed(123)
    got = sampler._CAPI_sample_node_classifiction(_cuda(seeds), fan_out, replace)
    exp = O.node_classification_sample(seeds, indptr, indices, fan_out, replace,
                                       O.launch_seeds(123, len(fan_out)), probs=probs)
    for (gs, gf, gr, gc), (es, ef, er, ec) in zip(got, exp):
        assert np.array_equal(gf.cpu().numpy(), ef)
        assert np.array_equal(gr.cpu().numpy(), er)
        assert np.array_equal(gc.cpu().numpy(), ec)


def test_pinned_tensor_outlives_caller_reference(dgs):
    """A tensor registered by _CAPI_tensor_pin_memory stays allocated while registered (the
    caller dropping it must not leave a registration over memory the allocator reuses), and
    _CAPI_tensor_unpin_memory releases it."""
    t = torch.arange(1 << 16, dtype=torch.int64)
    dgs.ops._CAPI_tensor_pin_memory(t)
    p = t.data_ptr()
    assert t.is_pinned()
    del t
    for _ in range(8):  # host allocations + device round trips that could reuse the range
        h = torch.randn(1 << 16)
        assert torch.equal(h.cuda().cpu(), h)
    kept = dgs.ops._registered[p][0]
    assert kept.data_ptr() == p and int(kept[-1]) == (1 << 16) - 1
    dgs.ops._CAPI_tensor_unpin_memory(kept)
    assert p not in dgs.ops._registered


def test_standalone_ops_on_two_streams(dgs):
    """The standalone ops keep their scratch per stream and the deterministic heat op its
    accumulator per call: heat on one stream interleaved with relabel + neighbour sampling on
    another (two threads) gives exactly what each gives alone."""
    import threading
    indptr, indices, probs = _hub_graph(2, giant=False)
    n = indptr.size - 1
    ip, ix = _cuda(indptr), _cuda(indices)
    heat = _cuda(np.random.default_rng(1).random(n).astype(np.float32))
    hseeds = _cuda(np.random.default_rng(2).permutation(n)[:300])
    rng = np.random.default_rng(4)
    maps = [_cuda(rng.integers(0, 300, 4000)), _cuda(rng.integers(0, 600, 9000))]
    sseeds = _cuda(rng.integers(0, n, 200))
    reps = 6

    def heat_op():
        return dgs.ops._CAPI_compute_frontier_heat(hseeds, ip, ix, heat, 5, 0,
                                                   deterministic=True)

    def other_ops():
        u, rel = dgs.ops._CAPI_cuda_sampled_tensor_relabel(maps, maps)
        r, c = dgs.ops._CAPI_cuda_sample_neighbors(sseeds, ip, ix, 10, False)
        return [u] + list(rel) + [r, c]

    exp_h = heat_op()
    dgs.ops._CAPI_set_random_seed(8)
    exp_o = [other_ops() for _ in range(reps)]
    torch.cuda.synchronize()
    got_h, got_o = [None] * reps, [None] * reps

    def run(fn, out, seed):
        st = torch.cuda.Stream()
        with torch.cuda.stream(st):
            if seed is not None:
                dgs.ops._CAPI_set_random_seed(seed)
            for i in range(reps):
                out[i] = fn()
            st.synchronize()

    ths = [threading.Thread(target=run, args=(heat_op, got_h, None)),
           threading.Thread(target=run, args=(other_ops, got_o, 8))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    for h in got_h:
        assert torch.equal(h, exp_h)
    for g, e in zip(got_o, exp_o):
        for a, b in zip(g, e):
            assert torch.equal(a, b)


def test_services_over_one_pageable_tensor_are_independent(dgs):
    """Two services over one pageable host tensor: each holds its own library-owned copy of what
    it reads (round 6: pageable caller memory is never registered), so destroying the first
    leaves the second exact, and no registration exists at any point."""
    import gc
    rng = np.random.default_rng(4)
    data = torch.from_numpy(rng.standard_normal((2000, 64)).astype(np.float32))
    base = dgs.ops._host_memory_state()
    a = dgs.classes.P2PCacheFeatureServer(data, torch.tensor([5]), 0)
    b = dgs.classes.P2PCacheFeatureServer(data, torch.tensor([9]), 0)
    st = dgs.ops._host_memory_state()
    assert st["registrations"] == base["registrations"]  # (pins of earlier tests may live on)
    # partly cached: each keeps a pinned mirror of the matrix for its host rows
    assert st["mirrors"] == base["mirrors"] + 2
    assert st["mirror_bytes"] == base["mirror_bytes"] + 2 * data.numel() * 4
    assert not data.is_pinned()
    q = rng.integers(0, 2000, 4096)
    exp = O.index_select(data.numpy(), q)
    assert np.array_equal(a._CAPI_get_feature(_cuda(q)).cpu().numpy(), exp)
    del a
    gc.collect()
    torch.cuda.synchronize()
    assert np.array_equal(b._CAPI_get_feature(_cuda(q)).cpu().numpy(), exp)
    del b
    gc.collect()
    assert dgs.ops._host_memory_state() == base
    c = dgs.classes.P2PCacheFeatureServer(data, torch.tensor([1]), 0)
    assert np.array_equal(c._CAPI_get_feature(_cuda(q)).cpu().numpy(), exp)


def test_unpin_keeps_a_live_service_mapped(dgs):
    """A service over a _CAPI_tensor_pin_memory tensor reads it in place, holding a reference on
    the pin: unpinning the tensor while the server reads it leaves the server's view mapped, and
    the registration goes with the server."""
    import gc
    rng = np.random.default_rng(6)
    data = torch.from_numpy(rng.standard_normal((1500, 32)).astype(np.float32))
    dgs.ops._CAPI_tensor_pin_memory(data)
    fs = dgs.classes.P2PCacheFeatureServer(data, torch.tensor([3]), 0)
    mirrors = dgs.ops._host_memory_state()["mirrors"]

    def mine():
        return [(r["base"], r["refs"], r["pins"]) for r in dgs.ops._host_registrations()
                if r["base"] == data.data_ptr()]
    assert mine() == [(data.data_ptr(), 2, 1)]
    dgs.ops._CAPI_tensor_unpin_memory(data)
    gc.collect()
    assert mine() == [(data.data_ptr(), 1, 0)]
    assert dgs.ops._host_memory_state()["mirrors"] == mirrors  # in place, no copy
    q = rng.integers(0, 1500, 2048)
    assert np.array_equal(fs._CAPI_get_feature(_cuda(q)).cpu().numpy(),
                          O.index_select(data.numpy(), q))
    del fs
    gc.collect()
    assert mine() == []


def test_services_over_views_of_one_buffer(dgs):
    """Services over different views of one pageable buffer (data[:k], data, data[k:]) copy their
    own ranges: destroying the first leaves the others byte-exact, with no registration."""
    import gc
    rng = np.random.default_rng(8)
    data = torch.from_numpy(rng.standard_normal((3000, 48)).astype(np.float32))
    k = 1000
    before = dgs.ops._host_memory_state()["registrations"]
    a = dgs.classes.P2PCacheFeatureServer(data[:k], torch.tensor([2]), 0)
    b = dgs.classes.P2PCacheFeatureServer(data, torch.tensor([7]), 0)
    c = dgs.classes.P2PCacheFeatureServer(data[k:], torch.tensor([0]), 0)
    assert dgs.ops._host_memory_state()["registrations"] == before
    qa, qb = rng.integers(0, k, 2048), rng.integers(0, 3000, 4096)
    assert np.array_equal(a._CAPI_get_feature(_cuda(qa)).cpu().numpy(),
                          O.index_select(data[:k].numpy(), qa))
    del a
    gc.collect()
    torch.cuda.synchronize()
    assert np.array_equal(b._CAPI_get_feature(_cuda(qb)).cpu().numpy(),
                          O.index_select(data.numpy(), qb))
    qc = rng.integers(0, 3000 - k, 2048)
    assert np.array_equal(c._CAPI_get_feature(_cuda(qc)).cpu().numpy(),
                          O.index_select(data[k:].numpy(), qc))


def test_c_abi_registration_rules(dgs):
    """At the C ABI: a range that only partly lies in a pin is refused (no unreferenced, partly
    unmapped view); an unregister must name a pointer that dgs_host_register pinned, and a
    contained range shares the registration."""
    import ctypes
    from dgs._lib import lib
    buf = torch.zeros(1 << 16, dtype=torch.uint8)
    base = (buf.data_ptr() + 4095) // 4096 * 4096 + 4096  # page aligned, inside buf

    def mine():
        return [(r["base"], r["bytes"], r["refs"], r["pins"]) for r in dgs.ops._host_registrations()
                if buf.data_ptr() <= r["base"] < buf.data_ptr() + buf.numel()]
    assert lib.dgs_host_register(ctypes.c_void_p(base), 4096) == 0
    # starts inside the registration, ends past it
    assert lib.dgs_host_register(ctypes.c_void_p(base + 1024), 8192) != 0
    assert b"overlaps" in lib.dgs_last_error()
    # a service over such a range is refused the same way
    with pytest.raises(RuntimeError, match="overlaps"):
        _raw_feature_server(base + 1024, 256, 32)
    # disjoint bytes on one page: two registrations, as the reference's cudaHostRegister of
    # neighbouring tensors (HIP locks the shared page for each; tests/test_host_pages_gpu.py
    # copies through such pages)
    q = base + 3 * 4096
    assert lib.dgs_host_register(ctypes.c_void_p(q), 100) == 0
    assert lib.dgs_host_register(ctypes.c_void_p(q + 200), 100) == 0
    assert lib.dgs_host_unregister(ctypes.c_void_p(q)) == 0
    assert lib.dgs_host_unregister(ctypes.c_void_p(q + 200)) == 0
    # the page after the first pin is free
    assert lib.dgs_host_register(ctypes.c_void_p(base + 4096), 4096) == 0
    assert lib.dgs_host_unregister(ctypes.c_void_p(base + 4096)) == 0
    # contained: shares, and needs its own unregister
    assert lib.dgs_host_register(ctypes.c_void_p(base + 512), 1024) == 0
    assert mine() == [(base, 4096, 2, 1)]
    assert lib.dgs_host_unregister(ctypes.c_void_p(base + 7)) != 0  # never pinned
    assert lib.dgs_host_unregister(ctypes.c_void_p(base + 512)) == 0
    assert lib.dgs_host_unregister(ctypes.c_void_p(base + 512)) != 0  # already released
    assert lib.dgs_host_unregister(ctypes.c_void_p(base)) == 0
    assert mine() == []
    # everything released: the larger range registers cleanly now
    assert lib.dgs_host_register(ctypes.c_void_p(base + 1024), 8192) == 0
    assert lib.dgs_host_unregister(ctypes.c_void_p(base + 1024)) == 0
    dgs.ops._check_async_errors()  # no failed unregister was recorded


def _raw_feature_server(ptr, rows, row_bytes):
    import ctypes
    from dgs._lib import check, lib
    h = ctypes.c_void_p()
    nids = torch.tensor([0], dtype=torch.int64)
    check(lib.dgs_feature_server_create(ctypes.c_void_p(ptr), rows, row_bytes,
                                        ctypes.c_void_p(nids.data_ptr()), 1, 0, ctypes.byref(h)))
    lib.dgs_feature_server_destroy(h)


@pytest.mark.parametrize("mode", [[], ["--loader"], ["--ops"]])
def test_random_sweep(mode):
    """tools/parity_sweep.py for a few seconds per mode: random graphs / caches / fan-outs through
    the synchronous call, the loader (with features) and the standalone ops, all exact."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "tools", "parity_sweep.py"),
                        "--seconds", "6", "--seed", "21"] + mode,
                       capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert " 0 mismatches" in p.stdout, p.stdout[-2000:]
