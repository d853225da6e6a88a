"""Randomised multi-rank parity sweep: W ranks (torchrun, gloo setup collectives through
dgs.ops._CAPI_set_host_comm, every rank on cuda:0 of one box) build the same random graph and
services each case, with a random cache placement over the ranks -- each node cached by no rank
(read from the pinned host mirror), one rank, or several (the reference's local-first rotation
picks the copy) -- and each rank checks its own sampled blocks against the oracle and its gathered
features against a host index.  Results do not depend on placement, so every rank must match.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29533 tools/mr_sweep.py [--seconds 200] [--seed 1]
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
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=200.0)
    ap.add_argument("--cases", type=int, default=100000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--full-cache", action="store_true",
                    help="every rank caches every node (no host mirror, no peer reads)")
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    import dgs
    from DistGNN.dataloading.synthetic import degree_probs, rmat_csc_numpy
    from oracle import oracle as O
    dgs.ops._CAPI_set_host_comm()
    rng = np.random.default_rng(a.seed)     # identical on every rank: the same cases
    mine = np.random.default_rng(1000 + rank)  # this rank's own seed batches
    t0 = time.time()
    done = bad = 0
    while done < a.cases:
        # every rank stops at the same case (the services' constructors are collective)
        stop = torch.tensor([time.time() - t0 > a.seconds], dtype=torch.int32)
        dist.all_reduce(stop, op=dist.ReduceOp.MAX)
        if stop.item():
            break
        scale, ef = int(rng.integers(8, 14)), int(rng.integers(1, 20))
        indptr, indices = rmat_csc_numpy(scale, ef, seed=int(rng.integers(1 << 30)))
        n = indptr.size - 1
        bias = bool(rng.random() < 0.4)
        probs = degree_probs(indptr, indices) if bias else None
        holders = rng.integers(0, 1 << world, n)  # bit r: node cached on rank r
        cache = np.nonzero((holders >> rank) & 1)[0]
        if cache.size == 0:
            cache = np.array([rank % n])
        fcache = np.nonzero((rng.integers(0, 1 << world, n) >> rank) & 1)[0]
        if fcache.size == 0:
            fcache = np.array([0])
        if a.full_cache:
            cache = fcache = np.arange(n)
        L = int(rng.integers(1, 4))
        fan_out = [int(rng.integers(1, 33 if bias else 41)) for _ in range(L)]
        replace = bool(rng.random() < 0.3)
        d = int(rng.choice([1, 7, 100]))
        feats = rng.standard_normal((n, d)).astype(np.float32)
        s = dgs.classes.P2PCacheSampler(torch.from_numpy(indptr), torch.from_numpy(indices),
                                        torch.from_numpy(probs) if bias else torch.Tensor(),
                                        torch.from_numpy(cache), 0)
        fs = dgs.classes.P2PCacheFeatureServer(torch.from_numpy(feats), torch.from_numpy(fcache),
                                               0)
        seeds = mine.integers(0, n, int(mine.integers(1, 1500)))
        ls = int(mine.integers(1, 1 << 40))
        dgs.ops._CAPI_set_random_seed(ls)
        got = s._CAPI_sample_node_classifiction(torch.from_numpy(seeds).cuda(), fan_out, replace)
        exp = O.node_classification_sample(seeds, indptr, indices, fan_out, replace,
                                           O.launch_seeds(ls, L), probs=probs)
        ok = len(got) == len(exp) and all(
            np.array_equal(g.cpu().numpy(), e) for gh, eh in zip(got, exp) for g, e in zip(gh, eh))
        x = fs._CAPI_get_feature(got[-1][1])
        ok = ok and np.array_equal(x.cpu().numpy(), feats[exp[-1][1]])
        torch.cuda.synchronize()
        del s, fs  # collective destructors, in the same order on every rank
        done += 1
        if not ok:
            bad += 1
            print(f"[rank {rank}] MISMATCH case {done}: scale {scale} ef {ef} bias {bias} "
                  f"replace {replace} fan_out {fan_out} cache {cache.size} fcache {fcache.size} "
                  f"seeds {seeds.size} seed {ls}", flush=True)
        if rank == 0 and done % 20 == 0:
            print(f"[mr-sweep] {done} cases, {time.time() - t0:.0f} s", flush=True)
        if done % 500 == 0:  # process resources over the cases (leak watch)
            free, _ = torch.cuda.mem_get_info()
            print(f"[mr-sweep] rank {rank} after {done} cases: {len(os.listdir('/proc/self/fd'))} "
                  f"open fds, {free / 2**30:.2f} GiB free on the device", flush=True)
    dgs.ops._check_async_errors()
    tot = torch.tensor([done, bad], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        print(f"multi-rank sweep: world {world}, {done} cases per rank, {int(tot[1])} mismatches "
              f"over all ranks, seed {a.seed}, {time.time() - t0:.0f} s", flush=True)
    dist.destroy_process_group()
    sys.exit(1 if int(tot[1]) else 0)


if __name__ == "__main__":
    main()
