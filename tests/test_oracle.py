"""Pins the CPU oracle (oracle/) against known answers and independent restatements.

Anchors, in order of strength:
  1. Random123 Philox4x32-10 published known answers; torch's header-only Philox engine
     streams and libstdc++'s std::mt19937_64 outputs (tests/golden/rng_kat.json, made by
     tests/golden/make_golden.py from tests/golden/gen_rng_kat.cpp).
  2. Known answers hand-derived from the reference's own tests (reference_kats.json).
  3. Literal pure-Python restatements of the reference kernels' thread loops
     (rowwise_sampling.cu:47-141, rowwise_sampling_bias.cu:62-224) on small inputs --
     written independently of the C oracle's reorganised loops.
  4. Structural invariants (hypothesis) and the committed oracle regression vectors.
"""
import json
import os

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from oracle import oracle as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


# ------------------------------------------------------------------ 1. RNG anchors
def test_philox_random123_kats():
    for kat in _load("rng_kat.json")["random123_philox4x32_10"]:
        assert list(O.philox4x32_10(kat["ctr"], kat["key"])) == kat["out"]


def test_curand_stream_matches_torch_philox_engine():
    for case in _load("rng_kat.json")["philox"]:
        got = O.curand_stream(case["seed"], case["subsequence"], case["offset_words"],
                              len(case["out"]))
        assert list(got) == case["out"], case


def test_curand_skipahead_word_offsets():
    # skipahead(offset) counts 32-bit words: offset o must equal dropping o words.
    full = O.curand_stream(99, 3, 0, 24)
    for off in range(0, 9):
        assert list(O.curand_stream(99, 3, off, 8)) == list(full[off:off + 8])


def test_philox_draw_is_jth_curand():
    s = O.curand_stream(0xABCDEF, 77, 0, 40)
    for j in range(40):
        assert O.philox_draw(0xABCDEF, 77, j) == s[j]


def test_curand_uniform_definition():
    raw = O.curand_stream(5, 6, 0, 64)
    uni = O.curand_stream(5, 6, 0, 64, uniform=True)
    ref = raw.astype(np.float32) * np.float32(2.0 ** -32) + np.float32(2.0 ** -33)
    assert np.array_equal(uni, ref.astype(np.float32))
    assert (uni > 0).all() and (uni <= 1).all()


def test_mt19937_64_launch_seeds():
    kat = _load("rng_kat.json")
    for case in kat["mt19937_64"]:
        assert [str(x) for x in O.launch_seeds(case["seed"], len(case["out"]))] == case["out"]
    g = O.MT64(5489)
    for _ in range(9999):
        g.next()
    assert str(g.next()) == kat["mt19937_64_10000th_default_seed"]


def test_log2f_accuracy_and_monotone():
    u = np.sort(np.random.default_rng(0).random(4000).astype(np.float32))
    u = u[u > 0]
    got = np.array([O.log2f(float(x)) for x in u], dtype=np.float64)
    np.testing.assert_allclose(got, np.log2(u.astype(np.float64)), rtol=2e-7, atol=2e-7)
    assert O.log2f(1.0) == 0.0
    assert O.ares_key(0.5, 0.0) == float("-inf")
    assert O.ares_key(0.5, 2.0) == -0.5


# ------------------------------------------------------------------ 2. reference KATs
def test_reference_extract_kat():
    k = _load("reference_kats.json")
    g, e = k["toy_graph"], k["extract"]
    sub = O.extract_indptr(e["cache_nids"], g["indptr"])
    assert list(sub) == e["sub_indptr"]
    assert list(O.extract_edge_data(e["cache_nids"], g["indptr"], sub,
                                    np.array(g["indices"]))) == e["sub_indices"]
    np.testing.assert_array_equal(
        O.extract_edge_data(e["cache_nids"], g["indptr"], sub,
                            np.array(g["probs"], np.float32)),
        np.array(e["sub_probs"], np.float32))


def test_reference_p2p_server_kat():
    k = _load("reference_kats.json")
    for nids, exp in zip(k["p2p_server"]["rank_cache_nids"], k["p2p_server"]["rank_sub_indptr"]):
        assert list(O.extract_indptr(nids, k["toy_graph"]["indptr"])) == exp


def test_reference_feature_server_kat():
    k = _load("reference_kats.json")["feature_server"]
    feat = np.arange(100, dtype=np.float32).reshape(10, 10)
    np.testing.assert_array_equal(O.index_select(feat, k["query"]),
                                  np.array(k["expected"], np.float32))


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("replace", [False, True])
def test_reference_sampler_kat(bias, replace):
    k = _load("reference_kats.json")
    g, s = k["toy_graph"], k["sampler"]
    for seed in range(20):
        res = O.node_classification_sample(s["seeds"], g["indptr"], g["indices"], s["fan_out"],
                                           replace, O.launch_seeds(seed, 2),
                                           probs=g["probs"] if bias else None)
        seeds0, frontier0, row0, col0 = res[0]
        assert list(frontier0[:3]) == s["frontier_prefix"]
        # seed 3 has degree 0; seeds 0 and 5 get exactly 2 picks each
        picked = {}
        for r, c in zip(row0, col0):
            picked.setdefault(int(seeds0[r]), []).append(int(frontier0[c]))
        assert set(picked) == {0, 5}
        for nid, cols in picked.items():
            assert len(cols) == 2
            assert set(cols) <= set(s["neighbours"][str(nid)])
            if not replace:
                assert len(set(cols)) == 2


# ------------------------------------------------------------------ 3. literal restatements
class _Curand:
    """Stateful curand Philox stream restated from curand_kernel.h, in pure Python."""

    def __init__(self, seed, sub):
        self.seed, self.sub, self.n = seed, sub, 0

    def next(self):
        v = O.philox_draw(self.seed, self.sub, self.n)
        self.n += 1
        return v

    def uniform(self):
        return np.float32(np.float32(self.next()) * np.float32(2.0 ** -32)
                          + np.float32(2.0 ** -33))


def _py_uniform_k2(seeds, indptr, indices, k, launch_seed):
    """rowwise_sampling.cu:47-104, thread-by-thread (grid = S, block = 128)."""
    S = len(seeds)
    rows, cols = [], []
    for r, row in enumerate(seeds):
        b, e = indptr[row], indptr[row + 1]
        deg = e - b
        if deg <= k:
            rows += [row] * deg
            cols += list(indices[b:e])
            continue
        slot = list(range(k))
        for t in range(128):
            rng = _Curand((launch_seed * S + r) % (1 << 64), t)
            idx = k + t
            while idx < deg:
                num = rng.next() % (idx + 1)
                if num < k:
                    slot[num] = max(slot[num], idx)
                idx += 128
        rows += [row] * k
        cols += [indices[b + x] for x in slot]
    return np.array(rows, np.int64), np.array(cols, np.int64)


def _py_uniform_k3(seeds, indptr, indices, k, launch_seed):
    """rowwise_sampling.cu:106-141."""
    S = len(seeds)
    rows, cols = [], []
    for r, row in enumerate(seeds):
        b, e = indptr[row], indptr[row + 1]
        deg = e - b
        if deg == 0:
            continue
        out = [None] * k
        for t in range(128):
            rng = _Curand((launch_seed * S + r) % (1 << 64), t)
            for idx in range(t, k, 128):
                out[idx] = indices[b + rng.next() % deg]
        rows += [row] * k
        cols += out
    return np.array(rows, np.int64), np.array(cols, np.int64)


def _py_bias(seeds, indptr, indices, probs, k, replace, launch_seed):
    """rowwise_sampling_bias.cu:62-224 with the DGS-AMD A-Res key (see dgs_oracle.h)."""
    S = len(seeds)
    G = (S + 15) // 16
    offs = [0]
    for row in seeds:
        deg = indptr[row + 1] - indptr[row]
        offs.append(offs[-1] + ((0 if deg == 0 else k) if replace else min(deg, k)))
    rows = [None] * offs[-1]
    cols = [None] * offs[-1]
    for blk in range(G):
        key = (launch_seed * G + blk) % (1 << 64)
        for w in range(4):
            lanes = [_Curand(key, (4 * w + l) if replace else (32 * w + l)) for l in range(32)]
            for r in range(16 * blk + w, min(16 * blk + 16, S), 4):
                row = seeds[r]
                b, e = indptr[row], indptr[row + 1]
                deg = e - b
                o = offs[r]
                if not replace:
                    if deg > k:
                        keys = [None] * deg
                        for l in range(32):
                            for i in range(l, deg, 32):
                                keys[i] = O.ares_key(float(lanes[l].uniform()),
                                                     float(probs[b + i]))
                        order = sorted(range(deg), key=lambda i: (-keys[i], i))[:k]
                        for j, i in enumerate(order):
                            rows[o + j], cols[o + j] = row, indices[b + i]
                    else:
                        for i in range(deg):
                            rows[o + i], cols[o + i] = row, indices[b + i]
                elif deg > 0:
                    cdf = np.zeros(deg, np.float32)
                    agg = np.float32(0)
                    for base in range(0, ((deg - 1) // 32 + 1) * 32, 32):
                        v = [np.float32(probs[b + base + l]) if base + l < deg else np.float32(0)
                             for l in range(32)]
                        v[0] = np.float32(v[0] + agg)
                        v = [np.float32(max(x, np.float32(0))) for x in v]
                        for s in range(5):
                            off = 1 << s
                            v = [np.float32(v[l - off] + v[l]) if l >= off else v[l]
                                 for l in range(32)]
                        agg = v[31]
                        for l in range(32):
                            if base + l < deg:
                                cdf[base + l] = v[l]
                    for l in range(32):
                        for idx in range(l, k, 32):
                            rnd = np.float32(lanes[l].uniform() * cdf[deg - 1])
                            item = min(int(np.searchsorted(cdf, rnd, side="right")), deg - 1)
                            rows[o + idx], cols[o + idx] = row, indices[b + item]
    return np.array(rows, np.int64), np.array(cols, np.int64)


def _small_graph(seed=3, n=64, maxdeg=300):
    rng = np.random.default_rng(seed)
    degs = rng.integers(0, maxdeg, n)
    degs[:4] = [0, 1, 5, 129]
    indptr = np.concatenate([[0], np.cumsum(degs)]).astype(np.int64)
    indices = rng.integers(0, n, indptr[-1]).astype(np.int64)
    probs = rng.random(indptr[-1]).astype(np.float32)
    probs[::7] = 0.0
    return indptr, indices, probs


@pytest.mark.parametrize("k", [1, 5, 15, 130])
def test_uniform_noreplace_matches_literal(k):
    indptr, indices, _ = _small_graph()
    seeds = np.random.default_rng(k).permutation(64)[:24]
    for ls in O.launch_seeds(k, 2):
        exp = _py_uniform_k2(list(seeds), indptr, indices, k, ls)
        got = O.sample_uniform(seeds, indptr, indices, k, False, ls)
        np.testing.assert_array_equal(got[0], exp[0])
        np.testing.assert_array_equal(got[1], exp[1])


@pytest.mark.parametrize("k", [1, 5, 130, 300])
def test_uniform_replace_matches_literal(k):
    indptr, indices, _ = _small_graph()
    seeds = np.random.default_rng(k).permutation(64)[:24]
    ls = O.launch_seeds(k + 1, 1)[0]
    exp = _py_uniform_k3(list(seeds), indptr, indices, k, ls)
    got = O.sample_uniform(seeds, indptr, indices, k, True, ls)
    np.testing.assert_array_equal(got[0], exp[0])
    np.testing.assert_array_equal(got[1], exp[1])


@pytest.mark.parametrize("replace", [False, True])
@pytest.mark.parametrize("k", [1, 4, 32])
def test_bias_matches_literal(replace, k):
    indptr, indices, probs = _small_graph(seed=5, maxdeg=90)
    seeds = np.random.default_rng(k).permutation(64)[:37]
    ls = O.launch_seeds(k + 11, 1)[0]
    exp = _py_bias(list(seeds), indptr, indices, probs, k, replace, ls)
    got = O.sample_bias(seeds, indptr, indices, probs, k, replace, ls)
    np.testing.assert_array_equal(got[0], exp[0])
    np.testing.assert_array_equal(got[1], exp[1])


# ------------------------------------------------------------------ 4. invariants
@settings(max_examples=40, deadline=None)
@given(st.integers(0, 2 ** 64 - 1), st.integers(1, 40), st.booleans(), st.booleans())
def test_sampler_invariants(launch_seed, k, replace, bias):
    indptr, indices, probs = _small_graph(seed=9, maxdeg=60)
    seeds = np.arange(0, 64, 3)
    if bias:
        row, col = O.sample_bias(seeds, indptr, indices, probs, k, replace, launch_seed)
    else:
        row, col = O.sample_uniform(seeds, indptr, indices, k, replace, launch_seed)
    degs = indptr[seeds + 1] - indptr[seeds]
    exp_nnz = int(np.where(degs > 0, k, 0).sum()) if replace else int(np.minimum(degs, k).sum())
    assert row.size == exp_nnz
    pos = 0
    for s, d in zip(seeds, degs):
        n = (k if d > 0 else 0) if replace else min(d, k)
        assert (row[pos:pos + n] == s).all()
        nb = indices[indptr[s]:indptr[s + 1]]
        assert np.isin(col[pos:pos + n], nb).all()
        pos += n


@settings(max_examples=40, deadline=None)
@given(st.lists(st.integers(0, 50), min_size=0, max_size=60),
       st.lists(st.integers(0, 50), min_size=0, max_size=60))
def test_relabel_semantics(a, b):
    uniq, (ra, rb) = O.relabel([a, b], [a, b])
    first = []
    for x in a + b:
        if x not in first:
            first.append(x)
    assert list(uniq) == first
    assert list(ra) == [first.index(x) for x in a]
    assert list(rb) == [first.index(x) for x in b]


def test_relabel_missing_is_minus_one():
    uniq, (r,) = O.relabel([[5, 6]], [[6, 7, 5]])
    assert list(uniq) == [5, 6] and list(r) == [1, -1, 0]


def test_node_classification_structure():
    z = np.load(os.path.join(GOLD, "sampler_golden.npz"))
    indptr, indices = z["indptr"], z["indices"]
    res = O.node_classification_sample(z["seeds"][:64], indptr, indices, [15, 10, 5], False,
                                       [int(x) for x in z["launch_seeds"][:3]])
    for h, (s, f, r, c) in enumerate(res):
        assert np.array_equal(f[:s.size], s)          # frontier prefix == seeds
        assert len(set(f.tolist())) == f.size          # unique
        assert (r < s.size).all() and (c < f.size).all()
        if h + 1 < len(res):
            assert np.array_equal(res[h + 1][0], f)


def test_oracle_regression_vectors():
    z = np.load(os.path.join(GOLD, "sampler_golden.npz"))
    ls = [int(x) for x in z["launch_seeds"]]
    i = 0
    for k in (3, 5, 15, 40):
        for rep in (0, 1):
            r, c = O.sample_uniform(z["seeds"], z["indptr"], z["indices"], k, rep, ls[i % 16])
            assert np.array_equal(r, z[f"uniform_k{k}_r{rep}_row"])
            assert np.array_equal(c, z[f"uniform_k{k}_r{rep}_col"])
            r, c = O.sample_bias(z["seeds"], z["indptr"], z["indices"], z["probs"], k, rep,
                                 ls[i % 16])
            assert np.array_equal(r, z[f"bias_k{k}_r{rep}_row"])
            assert np.array_equal(c, z[f"bias_k{k}_r{rep}_col"])
            i += 1


def test_openmp_uniform_equals_serial():
    z = np.load(os.path.join(GOLD, "sampler_golden.npz"))
    for rep in (False, True):
        a = O.sample_uniform(z["seeds"], z["indptr"], z["indices"], 10, rep, 1234)
        b = O.sample_uniform(z["seeds"], z["indptr"], z["indices"], 10, rep, 1234, nthreads=4)
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_heat_semantics():
    indptr, indices, probs = _small_graph(seed=1, n=32, maxdeg=20)
    probs = probs + np.float32(0.01)
    heat = np.random.default_rng(0).random(32).astype(np.float32)
    seeds = np.array([1, 2, 5, 9])
    fh = O.frontier_heat(seeds, indptr, indices, heat, 5)
    exp = np.zeros(32, np.float64)
    for s in seeds:
        d = indptr[s + 1] - indptr[s]
        for i in range(indptr[s], indptr[s + 1]):
            exp[indices[i]] += min(1.0, heat[s] * 5 / d)
    np.testing.assert_allclose(fh, exp, rtol=1e-5)
    fb = O.frontier_heat(seeds, indptr, indices, heat, 5, probs=probs)
    exp = np.zeros(32, np.float64)
    for s in seeds[:-1]:  # preprocess_heat.cu:107 drops the last seed
        b, e = indptr[s], indptr[s + 1]
        ps = probs[b:e].sum()
        for i in range(b, e):
            exp[indices[i]] += min(1.0, heat[s] * 5 * (probs[i] / ps))
    np.testing.assert_allclose(fb, exp, rtol=1e-5)


def test_cache_hashmap_restatement():
    """The reference's cache map (hashmap.h / hashmap.cu:15-77), sequential: capacity
    2 * _UpPower(total), every key found by SearchForPos, the local list's (idx, devid) win
    for a node cached on several ranks, the key set is the union of the lists."""
    import numpy as np
    from oracle import oracle as O
    assert [O.cache_hashmap_dir_size(t) for t in (1, 2, 3, 4, 5, 1000, 1024)] == \
        [4, 8, 8, 16, 16, 2048, 4096]
    # Murmur3 finalisers: fmix32 / fmix64 of 1 (published constants of the reference)
    assert O._murmur32(1) == 0x514E28B7
    assert O._murmur64(1) == 0xB456BCFC34C2CB2C
    rng = np.random.default_rng(3)
    for id_bytes in (8, 4):
        lists = [rng.choice(5000, 300, replace=False) for _ in range(3)]
        key, idx, dev = O.cache_hashmap(lists, local_rank=1, id_bytes=id_bytes)
        assert len(key) == O.cache_hashmap_dir_size(900)
        assert set(key[key >= 0].tolist()) == set(np.concatenate(lists).tolist())
        # the last list in insertion order (remote 2, 0 rotation from rank 1, then local 1)
        # holding a key writes its (idx, devid)
        want = {}
        for d in (2, 0, 1):
            for i, k in enumerate(lists[d].tolist()):
                want[k] = (i, d)
        for k, (i, d) in want.items():
            pos = O.cache_hashmap_find(key, k, id_bytes)
            assert pos >= 0 and key[pos] == k
            assert (idx[pos], dev[pos]) == (i, d)
