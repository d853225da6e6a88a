"""Benchmark of the DGS-AMD hot path (BASELINE.json metric: sampled edges/sec + feature-gather
GB/s, fan-out [15,10,5]).

One step = one training-loop data pass of the reference (example/graphsage/
node_classification.py:219-229): P2PCacheSampler._CAPI_sample_node_classifiction(seeds,
[15,10,5]) + P2PCacheFeatureServer._CAPI_get_feature(input nodes) +
ops._CAPI_cuda_index_select(labels, seeds), on a synthetic products-like RMAT graph (configs[1]:
uniform sampler + full-feature gather, d = 100, whole graph in HBM).  Inputs are resident in HBM
before the timed region.  Batches are prepared by DistGNN.dataloading.PrefetchLoader with
--depth batches in flight (each on its own stream, over one sampler and one feature server;
output identical to the sequential loop, which --depth 1 runs); the timed region holds exactly
K batches.  N > 1 (torchrun): every rank holds the graph (replicated, weak
scaling, independent replicas) and samples its own slice of the train nids; no collective
runs in the timed loop.  --shard caches node v on GPU v mod N instead (remote rows read
one-sided over xGMI through IPC-mapped peer memory).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--scale S --ef E]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--fan-out", type=str, default="15,10,5")
    p.add_argument("--scale", type=int, default=21)   # products-like: 2,097,152 nodes
    p.add_argument("--ef", type=int, default=59)      # 123.7 M edges
    p.add_argument("--dim", type=int, default=100)
    p.add_argument("--shard", action="store_true",
                   help="cache node v on GPU v %% N (P2P over xGMI) instead of replicating")
    p.add_argument("--bias", action="store_true",
                   help="biased (degree-weighted) sampler: probs[e] = 1 + indeg(indices[e])")
    p.add_argument("--cache-frac", type=float, default=1.0,
                   help="cache only the ceil(f*N) highest in-degree nodes in HBM; every other "
                        "row is read zero-copy from pinned host memory (SURVEY 8(f) rank 2)")
    p.add_argument("--comm", choices=["gloo", "rccl"], default="gloo",
                   help="transport of the library's setup collectives in --shard mode")
    p.add_argument("--depth", type=int, default=3,
                   help="batches in flight (PrefetchLoader streams); 1 = the sequential loop")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--seed", type=int, default=20261015)
    return p.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # DGS_BENCH_SHARE_DEVICE=1 rehearses the N>1 flow on a 1-GPU box: every rank on cuda:0,
    # gloo process group (RCCL refuses two ranks on one device).
    share = os.environ.get("DGS_BENCH_SHARE_DEVICE") == "1"
    if share:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    import dgs
    from DistGNN.dataloading import PrefetchLoader, SeedGenerator
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    if world > 1 and args.shard:
        # setup collectives only (IPC handles, cache lists); the timed loop has none
        if args.comm == "rccl" and not share:
            from DistGNN.dist import create_communicator
            create_communicator(world)
        else:
            dgs.ops._CAPI_set_host_comm(dist.group.WORLD if share
                                        else dist.new_group(backend="gloo"))

    fan_out = [int(x) for x in args.fan_out.split(",")]
    dev = torch.device("cuda", local_rank)

    # ---------------- synthetic inputs (identical on every rank)
    t0 = time.time()
    indptr_d, indices_d = rmat_csc_torch(args.scale, args.ef, seed=args.seed, device=dev)
    N = indptr_d.numel() - 1
    E = indices_d.numel()
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats_d = torch.randn(N, args.dim, generator=gen, device=dev)
    labels_d = torch.randint(0, 47, (N,), generator=gen, device=dev)
    probs = torch.Tensor()
    hot = None
    if args.cache_frac < 1.0:  # hot set: highest in-degree first (ties by id), kept on host
        n_hot = max(1, int(math.ceil(args.cache_frac * N)))
        indeg = torch.bincount(indices_d, minlength=indptr_d.numel() - 1)
        hot = torch.sort(indeg, descending=True, stable=True).indices[:n_hot].cpu()
        del indeg
    if args.bias:  # degree-weighted, probs[e] = float32(1 + indeg(indices[e]))
        indeg = torch.bincount(indices_d, minlength=indptr_d.numel() - 1)
        probs = (1 + indeg[indices_d]).to(torch.float32).cpu()
        del indeg
    indptr, indices = indptr_d.cpu(), indices_d.cpu()
    feats, labels = feats_d.cpu(), labels_d.cpu()
    del indptr_d, indices_d, feats_d, labels_d
    torch.cuda.empty_cache()
    g2 = torch.Generator()
    g2.manual_seed(2)
    train = torch.randperm(N, generator=g2)[: N // 10]
    train_local = seed_slice(train, rank, world).to(dev)
    log(f"[bench] graph N={N} E={E} d={args.dim} built in {time.time() - t0:.1f}s")

    # ---------------- services: whole graph + all features in HBM (configs[1])
    if hot is not None:
        cache = hot[rank::world] if args.shard and world > 1 else hot
    elif args.shard and world > 1:
        cache = torch.arange(rank, N, world)
    else:
        cache = torch.arange(N)
    # which nodes any GPU holds (the rest are host rows), for the host-row share reported below
    cached_mask = torch.zeros(N, dtype=torch.bool, device=dev)
    cached_mask[(hot if hot is not None else torch.arange(N)).to(dev)] = True
    t0 = time.time()
    sampler = dgs.classes.P2PCacheSampler(indptr, indices, probs, cache, local_rank)
    server = dgs.classes.P2PCacheFeatureServer(feats, cache, local_rank)
    labels_dev = labels.to(dev)
    layout = server._layout()
    torch.cuda.synchronize()
    log(f"[bench] services ready in {time.time() - t0:.1f}s")
    dgs.ops._CAPI_set_random_seed(args.seed + rank)

    torch.manual_seed(1)
    loader = iter(SeedGenerator(train_local, args.batch, shuffle=True, drop_last=True))

    def next_seeds():
        nonlocal loader
        try:
            return next(loader)
        except StopIteration:
            loader = iter(SeedGenerator(train_local, args.batch, shuffle=True, drop_last=True))
            return next(loader)

    def step(seeds):
        """The sequential loop body.  The label gather depends only on the seeds: issued
        first, it runs while the host enters the sampler (the reference loop's order,
        node_classification.py:219-229, is sample -> features -> labels)."""
        y = dgs.ops._CAPI_cuda_index_select(labels_dev, seeds)
        blocks = sampler._CAPI_sample_node_classifiction(seeds, fan_out, False)
        x = server._CAPI_get_feature(blocks[-1][1])
        return blocks, x, y

    def batches_of(seed_batches):
        if args.depth == 1:
            return (step(s) for s in seed_batches)
        return PrefetchLoader(sampler, seed_batches, fan_out, server=server, labels=labels_dev,
                              depth=args.depth)

    for _ in batches_of([next_seeds() for _ in range(args.warmup)]):
        pass
    # the timed batches' seeds (views of the shuffled train set, as SeedGenerator yields them)
    timed = [next_seeds() for _ in range(args.steps)]
    it = batches_of(timed)  # worker threads start here; no batch is submitted before t0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # only the gather kernel is measured in the timed region: its workgroups stamp their own
    # start / end (no stream markers between the measured kernels)
    dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    seg0 = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)
    edges = rows = 0
    t0 = time.perf_counter()
    step_t = []
    for blocks, x, _ in it:
        step_t.append(time.perf_counter())
        edges += sum(b[2].numel() for b in blocks)
        rows += x.shape[0]
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    prof = dgs.ops.profile_read()
    # hipMalloc calls the caching allocator made inside the timed region (host stalls)
    mallocs = torch.cuda.memory_stats(dev).get("segment.all.allocated", 0) - seg0
    # host-side spacing of consecutive batches handed out by the loader (jitter diagnostics)
    gaps = np.diff(np.array([t0] + step_t)) * 1e3
    step_gaps = {"p10": float(np.percentile(gaps, 10)), "p50": float(np.median(gaps)),
                 "p90": float(np.percentile(gaps, 90)), "max": float(gaps.max())}
    # informational, outside the timed region: the sequential loop's latency per sample call
    # (host wall, sample + label select), its GPU span, and the feature gather on its own
    n_side = min(args.steps, 20)
    side_seeds = [next_seeds() for _ in range(n_side)]
    torch.cuda.synchronize()
    dgs.ops.profile_enable(dgs.ops.PROFILE_SAMPLE | dgs.ops.PROFILE_SELECT)
    ts = time.perf_counter()
    side_nids = []
    for s in side_seeds:
        dgs.ops._CAPI_cuda_index_select(labels_dev, s)
        side_nids.append(sampler._CAPI_sample_node_classifiction(s, fan_out, False)[-1][1])
    torch.cuda.synchronize()
    seq_ms = (time.perf_counter() - ts) * 1e3 / n_side
    side = dgs.ops.profile_read()
    # share of the gathered rows that are host rows, over the side pass's batches (the timed
    # loop keeps no batch alive: each one it held would pin its output buffers, and the
    # caching allocator would hipMalloc fresh ones inside the timed region)
    host_rows = sum(float((~cached_mask[n.long()]).sum()) / max(n.numel(), 1)
                    for n in side_nids) / max(len(side_nids), 1)
    dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    iso_rows = 0
    for n in side_nids:
        iso_rows += server._CAPI_get_feature(n).shape[0]
    torch.cuda.synchronize()
    iso = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    # SURVEY 8(d) metric (2) as defined there: algorithmic bytes / wall time of one synchronous
    # _CAPI_get_feature call (host launch + kernel + synchronisation), median over the side pass
    call_ms = []
    for n in side_nids:
        tc = time.perf_counter()
        server._CAPI_get_feature(n)
        torch.cuda.synchronize()
        call_ms.append((time.perf_counter() - tc) * 1e3)
    call_i = int(np.argsort(call_ms)[len(call_ms) // 2])
    call_gbps = (side_nids[call_i].numel() * (2 * args.dim * 4 + 8) / (call_ms[call_i] * 1e-3) / 1e9
                 if call_ms else 0.0)

    row_bytes = args.dim * 4
    gather_bytes = rows * (2 * row_bytes + 8)  # read row + write row + read nid
    elapsed, edges_all, rows_all, gbytes_all = reduce_over_ranks(
        dist, torch.device("cpu") if share else dev, elapsed, edges, rows, gather_bytes)

    # roofline of the dominant HBM kernel (feature gather), measured live with HIP events
    g_ms = prof["gather_ms"] / max(prof["gather_launches"], 1)
    g_bytes = gather_bytes / max(prof["gather_launches"], 1)
    achieved = g_bytes / (g_ms * 1e-3) / 1e9 if g_ms > 0 else 0.0
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "gather_pmc.json")
    if os.path.exists(pmc_path):
        try:
            pmc = json.load(open(pmc_path))
            if pmc.get("dim") == args.dim:
                traffic = pmc.get("hbm_bytes_per_row") * (rows / max(prof["gather_launches"], 1))
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(indptr, indices, probs if args.bias else None, feats, train, fan_out,
                           args)

    out = {
        "metric": "sampled edges/sec + feature-gather GB/s, fan-out [15,10,5]",
        "value": edges_all / elapsed,
        "unit": "sampled edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (RMAT a,b,c,d=.57,.19,.19,.05; randn f32 features; no OGB offline)",
        "config": {
            "workload": (f"products-like RMAT scale {args.scale} ef {args.ef} (N={N}, E={E}), "
                         f"{'biased (degree-weighted)' if args.bias else 'uniform'} sampler "
                         f"fan-out {fan_out} without replacement, B={args.batch} "
                         f"seeds/step/GPU, + full-feature gather d={args.dim} f32 + label gather; "
                         + (f"HBM cache of the {args.cache_frac:.0%} highest in-degree nodes "
                            f"({'sharded' if args.shard and world > 1 else 'replicated'}), "
                            "other rows zero-copy from pinned host" if hot is not None else
                            "graph sharded v%N over GPUs (P2P)" if args.shard and world > 1
                            else "whole graph + features in HBM on every GPU")),
            "fan_out": fan_out, "batch_per_gpu": args.batch, "num_nodes": N, "num_edges": E,
            "feat_dim": args.dim, "parallelism": f"dp{world} (seed-parallel)",
            "cache_frac": args.cache_frac,
            "pipeline_depth": args.depth,
        },
        "host_step_gap_ms": step_gaps,
        "allocator_mallocs_in_timed_region": mallocs,
        "host_row_share": host_rows,
        # host rows cross PCIe Gen5 x16 (63 GB/s spec): their read rate during the gather
        "gather_host_read_GBps": (host_rows * rows * row_bytes / (prof["gather_ms"] * 1e-3) / 1e9
                                  if prof["gather_ms"] > 0 else 0.0),
        "gather_GBps": achieved,
        "gather_GBps_wall": gbytes_all / elapsed / 1e9,
        "gather_GBps_sync_call": call_gbps,
        "sampled_edges_per_step": edges_all / args.steps,
        "gathered_rows_per_step": rows_all / args.steps,
        "gather_kernel_ms_per_step": prof["gather_ms"] / args.steps,
        "sample_span_ms_per_call": side["sample_ms"] / max(side["sample_calls"], 1),
        "sequential_sample_ms_per_call": seq_ms,
        "label_select_kernel_ms": side["select_ms"] / max(side["select_launches"], 1),
        "roofline": {
            "bound": "hbm",
            "kernel": ("k_gather<16, StridedSrc> (P2PCacheFeatureServer gather, computed row "
                       "addresses)" if layout >= 0 else
                       "k_gather<16, TableSrc> (P2PCacheFeatureServer gather, address table)"),
            "timing": ("device-side s_memrealtime stamps per workgroup (first workgroup start to "
                       "last workgroup end of each launch, 100 MHz wall clock) over the timed "
                       "region, where each gather shares the GPU with the sampling kernels of the "
                       "other batches in flight"),
            "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "bytes_per_launch": g_bytes, "avg_launch_ms": g_ms,
            "traffic": traffic,
        },
        # the same gather kernel with nothing running beside it (sequential side pass)
        "roofline_isolated": {
            "achieved": (iso_rows * (2 * args.dim * 4 + 8) / (iso["gather_ms"] * 1e-3) / 1e9
                         if iso["gather_ms"] > 0 else 0.0),
            "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": (iso_rows * (2 * args.dim * 4 + 8) / (iso["gather_ms"] * 1e-3) / 1e9
                     / HBM_PEAK_GBPS if iso["gather_ms"] > 0 else 0.0),
            "avg_launch_ms": iso["gather_ms"] / max(iso["gather_launches"], 1),
        },
        "cpu_baseline": cpu,
    }
    if rank == 0:
        print(json.dumps(out), flush=True)
    del sampler, server  # collective destructors (sharded mode) before the group goes away
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
        dist.destroy_process_group()


def reduce_over_ranks(dist, dev, elapsed, edges, rows, gather_bytes):
    """Job time = max over ranks (every rank ran the same K steps between barriers); work =
    sum over ranks.  dist is None for a single process."""
    if dist is None:
        return elapsed, float(edges), float(rows), float(gather_bytes)
    t = torch.tensor([elapsed, float(edges), float(rows), float(gather_bytes)],
                     dtype=torch.float64, device=dev)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(mx[0]), float(t[1]), float(t[2]), float(t[3])


def seed_slice(train, rank, world):
    """Train nids of this rank (node_classification.py:312-321: contiguous equal slices)."""
    per = (train.numel() + world - 1) // world
    return train[rank * per:(rank + 1) * per]


def host_info():
    """The box's CPU as the baseline ran on it (state the core count)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "usable_cpus": usable}


def cpu_baseline(indptr, indices, probs, feats, train, fan_out, args):
    """The oracle's OpenMP restatement on the host cores (DGL is not installed): row-wise
    sampling per hop (uniform, or biased when probs is given) + relabel + feature gather, same
    graph and batch size."""
    from oracle import oracle as O
    threads = int(os.environ.get("DGS_CPU_THREADS", "16"))
    ip, ix = indptr.numpy(), indices.numpy()
    pr = probs.numpy() if probs is not None else None
    fx = feats.numpy()
    rng = np.random.default_rng(1)
    seeds_all = train.numpy()
    edges = rows = batches = 0
    t0 = time.perf_counter()
    while True:
        seeds = seeds_all[rng.integers(0, seeds_all.size, args.batch)]
        cur = seeds
        for h, k in enumerate(reversed(fan_out)):
            if probs is None:
                r, c = O.sample_uniform(cur, ip, ix, k, False, 1000 + batches * 8 + h,
                                        nthreads=threads)
            else:
                r, c = O.sample_bias(cur, ip, ix, pr, k, False, 1000 + batches * 8 + h,
                                     nthreads=threads)
            uniq, (rr, cc) = O.relabel([cur, c], [r, c])
            edges += c.size
            cur = uniq
        x = O.index_select(fx, cur, nthreads=threads)
        rows += x.shape[0]
        batches += 1
        if time.perf_counter() - t0 > args.cpu_baseline_seconds:
            break
    dt = time.perf_counter() - t0
    # the CPU gather baseline proper is torch.index_select on the host feature
    # tensor with the same nids (here: the last batch's frontier, repeated for ~1 s)
    torch.set_num_threads(threads)
    nid = torch.from_numpy(np.ascontiguousarray(cur))
    reps, t1 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t1 < 1.0:
        torch.index_select(feats, 0, nid)
        reps += 1
    ts_gbps = reps * nid.numel() * (2 * args.dim * 4 + 8) / (time.perf_counter() - t1) / 1e9
    return {"value": edges / dt, "unit": "sampled edges/s", "cores": threads, "kind": "port",
            "host": host_info(),
            "gather_GBps": rows * (2 * args.dim * 4 + 8) / dt / 1e9,
            "gather_GBps_torch_index_select": ts_gbps,
            "sample": (f"{batches} batches of B={args.batch}, fan-out {fan_out}, same graph; "
                       f"oracle/dgs_oracle.c OpenMP {'biased' if probs is not None else 'uniform'} "
                       f"sampler ({threads} threads) + serial relabel "
                       f"+ OpenMP gather, {dt:.1f}s")}


if __name__ == "__main__":
    main()
