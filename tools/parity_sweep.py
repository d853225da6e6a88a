"""Randomised parity sweep of the node-classification sampler (GPU) against the oracle: random
RMAT graphs (scale 8 to --max-scale, edge factor 1-24) with planted hub rows, random cache
subsets (all, a fraction, one node), 1-3 hops of random fan-outs, with / without replacement,
uniform or weighted (degree weights or random weights with zeros), random seed batches with
repeats.  Every output tensor of every hop is compared exactly; a mismatch prints its
configuration.

    python tools/parity_sweep.py [--cases 300] [--seconds 240] [--seed 1] [--max-scale 14]
        [--max-batch 2048]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def graph(rng, max_scale=14):
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_numpy
    scale = int(rng.integers(8, max_scale + 1))
    ef = int(rng.integers(1, 25))
    indptr, indices = rmat_csc_numpy(scale, ef, seed=int(rng.integers(1 << 30)))
    n = indptr.size - 1
    # planted hub rows (appended): degrees around the samplers' limits and a few long rows
    extra = rng.choice([130, 144, 700, 1025, 2049, 4097, 8193, 30000], int(rng.integers(0, 4)))
    if extra.size:
        tails = [rng.integers(0, n, int(d)) for d in extra]
        indptr = np.concatenate([indptr, indptr[-1] + np.cumsum([t.size for t in tails])])
        indices = np.concatenate([indices] + tails)
    indptr = indptr.astype(np.int64)
    indices = indices.astype(np.int64)
    if rng.random() < 0.5:
        probs = degree_probs(indptr, indices)
    else:
        probs = (rng.random(indices.size) + 0.01).astype(np.float32)
        probs[rng.random(indices.size) < 0.05] = 0.0
    return indptr, indices, probs, scale, ef, extra.tolist()


def same(got, exp):
    return len(got) == len(exp) and all(
        np.array_equal(g.cpu().numpy(), e) for gh, eh in zip(got, exp) for g, e in zip(gh, eh))


def loader_case(dgs, O, rng, sampler, indptr, indices, probs, fan_out, replace, seeds, ls, cfg):
    """2-6 batches of the configuration's seeds through PrefetchLoader (random depth, a feature
    server over a random cache and row width): blocks against the oracle with the engine's launch
    seeds in submission order (L per batch), features against a host index."""
    from DistGNN.dataloading import PrefetchLoader
    n = indptr.size - 1
    L = len(fan_out)
    d = int(rng.choice([1, 3, 16, 100]))
    feats = rng.standard_normal((n, d)).astype(np.float32)
    fcache = np.arange(n) if rng.random() < 0.5 else rng.permutation(n)[: max(1, n // 3)]
    server = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(feats), torch.from_numpy(fcache),
                                               0)
    nb = int(rng.integers(2, 7))
    depth = int(rng.integers(1, 4))
    batches = [torch.from_numpy(np.roll(seeds, 7 * i)).cuda() for i in range(nb)]
    cfg.update(loader_batches=nb, depth=depth, dim=d, feat_cache=int(fcache.size))
    got = list(PrefetchLoader(sampler, batches, fan_out, replace=replace, server=server,
                              depth=depth))
    allseeds = O.launch_seeds(ls, L * nb)
    ok = len(got) == nb
    for i, (b, (blocks, x, _)) in enumerate(zip(batches, got)):
        exp = O.node_classification_sample(b.cpu().numpy(), indptr, indices, fan_out, replace,
                                           allseeds[L * i:L * (i + 1)], probs=probs)
        ok = ok and same(blocks, exp)
        ok = ok and np.array_equal(x.cpu().numpy(), feats[exp[-1][1]])
    del server
    return ok


def ops_case(dgs, O, rng, max_scale):
    """One random case of each standalone op."""
    indptr, indices, probs, scale, ef, extra = graph(rng, max_scale)
    n = indptr.size - 1
    idt = torch.int32 if rng.random() < 0.4 else torch.int64
    k = int(rng.integers(1, 41))
    replace = bool(rng.random() < 0.3)
    bias = bool(rng.random() < 0.4)
    if bias:
        k = min(k, 32)
    seeds = rng.integers(0, n, int(rng.integers(1, 3000)))
    ls = int(rng.integers(1, 1 << 40))
    cfg = dict(op="sample", scale=scale, ef=ef, extra=extra, ids=str(idt), k=k, replace=replace,
               bias=bias, seeds=int(seeds.size), seed=ls)
    dev = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(idt).cuda()  # noqa: E731
    dgs.ops._CAPI_set_random_seed(ls)
    l0 = O.launch_seeds(ls, 1)[0]
    if bias:
        row, col = dgs.ops._CAPI_cuda_sample_neighbors_bias(
            dev(seeds), dev(indptr), dev(indices), torch.from_numpy(probs).cuda(), k, replace)
        er, ec = O.sample_bias(seeds, indptr, indices, probs, k, replace, l0)
    else:
        row, col = dgs.ops._CAPI_cuda_sample_neighbors(dev(seeds), dev(indptr), dev(indices), k,
                                                       replace)
        er, ec = O.sample_uniform(seeds, indptr, indices, k, replace, l0)
    ok = (row.dtype == idt and np.array_equal(row.cpu().numpy().astype(np.int64), er) and
          np.array_equal(col.cpu().numpy().astype(np.int64), ec))
    if not ok:
        return False, cfg
    # relabel over arbitrary int64 keys (negative and above 2^32 too), 1-3 lists of each kind
    span = int(rng.choice([10, 1000, 1 << 20]))
    base = int(rng.integers(-(1 << 40), 1 << 40))
    maps = [base + rng.integers(0, span, int(rng.integers(0, 5000)))
            for _ in range(int(rng.integers(1, 4)))]
    reqs = [base + rng.integers(0, 2 * span, int(rng.integers(0, 5000)))
            for _ in range(int(rng.integers(1, 4)))]
    cfg = dict(op="relabel", span=span, base=base, maps=[m.size for m in maps],
               reqs=[r.size for r in reqs])
    u, rel = dgs.ops._CAPI_cuda_sampled_tensor_relabel([torch.from_numpy(m).cuda() for m in maps],
                                                      [torch.from_numpy(r).cuda() for r in reqs])
    eu, erel = O.relabel(maps, reqs)
    ok = np.array_equal(u.cpu().numpy(), eu) and all(
        np.array_equal(g.cpu().numpy(), e) for g, e in zip(rel, erel))
    if not ok:
        return False, cfg
    # index_select: int32 / int64 / float32 rows of random width, int32 / int64 ids
    vdt = [np.int32, np.int64, np.float32][int(rng.integers(3))]
    shape = (int(rng.integers(1, 5000)),) + tuple(int(x) for x in
                                                   rng.integers(1, 9, int(rng.integers(0, 3))))
    data = (rng.standard_normal(shape) * 1000).astype(vdt)
    nids = rng.integers(0, shape[0], int(rng.integers(0, 20000)))
    cfg = dict(op="index_select", dtype=str(vdt), shape=shape, n=int(nids.size), ids=str(idt))
    got = dgs.ops._CAPI_cuda_index_select(torch.from_numpy(data).cuda(),
                                          torch.from_numpy(nids).to(idt).cuda())
    return np.array_equal(got.cpu().numpy(), data[nids]), cfg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", type=int, default=300)
    ap.add_argument("--seconds", type=float, default=240.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--max-scale", type=int, default=14)
    ap.add_argument("--max-batch", type=int, default=2048)
    ap.add_argument("--ops", action="store_true",
                    help="sweep the standalone ops instead: _CAPI_cuda_sample_neighbors(_bias) "
                         "with int32 / int64 ids, _CAPI_cuda_sampled_tensor_relabel over "
                         "arbitrary int64 keys, _CAPI_cuda_index_select")
    ap.add_argument("--loader", action="store_true",
                    help="run 2-6 batches per configuration through PrefetchLoader (depth 1-3) "
                         "with a feature server, and check the features too")
    a = ap.parse_args()
    import dgs
    from oracle import oracle as O
    torch.cuda.set_device(0)
    rng = np.random.default_rng(a.seed)
    t0 = time.time()
    done = bad = 0
    counts = {"bias": 0, "replace": 0, "hops": [0, 0, 0]}
    while a.ops and done < a.cases and time.time() - t0 < a.seconds:
        ok, cfg = ops_case(dgs, O, rng, a.max_scale)
        done += 1
        if not ok:
            bad += 1
            print(f"MISMATCH {cfg}", flush=True)
        if done % 20 == 0:
            print(f"[sweep] {done} cases, {bad} mismatches, {time.time() - t0:.0f} s", flush=True)
    while not a.ops and done < a.cases and time.time() - t0 < a.seconds:
        indptr, indices, probs, scale, ef, extra = graph(rng, a.max_scale)
        n = indptr.size - 1
        bias = bool(rng.random() < 0.4)
        replace = bool(rng.random() < 0.3)
        L = int(rng.integers(1, 4))
        kmax = 32 if bias else 40
        fan_out = [int(rng.integers(1, kmax + 1)) for _ in range(L)]
        c = rng.random()
        if c < 0.4:
            cache = np.arange(n)
        elif c < 0.8:
            cache = rng.permutation(n)[: max(1, int(n * rng.random()))]
        else:
            cache = np.array([int(rng.integers(n))])
        B = int(rng.integers(1, a.max_batch + 1))
        seeds = rng.integers(0, n, B) if rng.random() < 0.5 else rng.permutation(n)[: min(B, n)]
        ls = int(rng.integers(1, 1 << 40))
        cfg = dict(scale=scale, ef=ef, extra=extra, bias=bias, replace=replace, fan_out=fan_out,
                   cache=int(cache.size), n=n, seeds=int(seeds.size), seed=ls)
        s = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                        torch.from_numpy(probs) if bias else torch.Tensor(),
                                        torch.from_numpy(cache), 0)
        dgs.ops._CAPI_set_random_seed(ls)
        if a.loader:
            ok = loader_case(dgs, O, rng, s, indptr, indices, probs if bias else None, fan_out,
                             replace, seeds, ls, cfg)
        else:
            got = s._CAPI_sample_node_classifiction(torch.from_numpy(seeds).cuda(), fan_out,
                                                    replace)
            exp = O.node_classification_sample(seeds, indptr, indices, fan_out, replace,
                                               O.launch_seeds(ls, L),
                                               probs=probs if bias else None)
            ok = same(got, exp)
        del s
        done += 1
        counts["bias"] += bias
        counts["replace"] += replace
        counts["hops"][L - 1] += 1
        if not ok:
            bad += 1
            print(f"MISMATCH {cfg}", flush=True)
        if done % 20 == 0:
            print(f"[sweep] {done} cases, {bad} mismatches, {time.time() - t0:.0f} s", flush=True)
    dgs.ops._check_async_errors()
    if a.ops:
        print(f"ops sweep: {done} cases (each: one sampling op, one relabel, one index_select), "
              f"{bad} mismatches, seed {a.seed}, {time.time() - t0:.0f} s")
    else:
        print(f"parity sweep: {done} cases ({counts['bias']} weighted, {counts['replace']} with "
              f"replacement, 1/2/3 hops {counts['hops']}), {bad} mismatches, seed {a.seed}, "
              f"{time.time() - t0:.0f} s")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
