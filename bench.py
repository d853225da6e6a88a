"""Benchmark of the DGS-AMD hot path (BASELINE.json metric: sampled edges/sec + feature-gather
GB/s, fan-out [15,10,5], 1/2/4/8 GPUs).

One step = one training-loop data pass of the reference (example/graphsage/
node_classification.py:219-229): P2PCacheSampler._CAPI_sample_node_classifiction(seeds,
[15,10,5]) + P2PCacheFeatureServer._CAPI_get_feature(input nodes) +
ops._CAPI_cuda_index_select(labels, seeds), on a synthetic products-like RMAT graph.  Inputs
are resident in HBM before the timed region.  Batches are prepared by
DistGNN.dataloading.PrefetchLoader with --depth batches in flight (each on its own stream, over
one sampler and one feature server; output identical to the sequential loop, which --depth 1
runs); the timed region holds exactly K batches per rank.

Workloads (--mode):
  replicated     configs[1] (the N = 1 default): whole graph + all features in every GPU's HBM.
  hot-shard      configs[2] (the N > 1 default): the graph structure in every GPU's HBM; a
                 hot-node feature cache (the --hot-frac highest in-degree nodes) on every GPU and
                 the other feature rows sharded v mod N behind the P2P feature server (remote
                 rows read one-sided over xGMI through IPC-mapped peer memory; setup collectives
                 over RCCL).  The reference's cache planner gives each GPU its hot nodes and pools
                 the rest (cache_value.py:65-150, 277-308).
  feature-shard  the same with no hot cache: every feature row sharded v mod N.
  shard          structure and features both sharded v mod N (neighbour lists read over xGMI
                 too: the configs[4] "gather + xGMI p2p" stress layout).
--cache-frac f < 1 keeps only the ceil(f*N) highest in-degree nodes in HBM (sharded by rank in
the sharded modes); every other row is read zero-copy from pinned host memory.

Launch: `python bench.py --gpus N` with no torchrun environment spawns N ranks itself (one
process per GPU, before any GPU call); under torchrun (WORLD_SIZE set) WORLD_SIZE must equal
--gpus.  With N > 1 local rank 0 builds the synthetic inputs once and every rank maps the same
host copy from /dev/shm (the reference shares one host copy through mp.spawn,
node_classification.py:325-328).  Every rank samples its own slice of the train nids; the timed
loop has no collective.  value = sampled edges of all ranks / max-over-ranks time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--scale S --ef E]
                       [--mode replicated|hot-shard|feature-shard|shard] [--hot-frac h]
                       [--bias] [--cache-frac f]
"""
import argparse
import gc
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# DGS_BENCH_PYDIR: another copy of the Python packages (same-box A/B of host-side changes)
sys.path.insert(0, os.environ.get("DGS_BENCH_PYDIR", os.path.join(ROOT, "dist-gnn_amd", "python")))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBPS = 153.0  # one xGMI link per peer
# the SURVEY 8(d) synthetic shapes by RMAT (scale, edge factor)
WORKLOADS = {(17, 9): "arxiv-like", (21, 59): "products-like", (27, 12): "papers100M-like",
             (26, 16): "RMAT-1B"}
CONFIG_OF_MODE = {"replicated": "configs[1]", "hot-shard": "configs[2]",
                  "feature-shard": "configs[2] without its hot cache",
                  "shard": "configs[4] layout"}


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=1000)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--fan-out", type=str, default="15,10,5")
    p.add_argument("--scale", type=int, default=21)   # products-like: 2,097,152 nodes
    p.add_argument("--ef", type=int, default=59)      # 123.7 M edges
    p.add_argument("--dim", type=int, default=100)
    p.add_argument("--mode", default="auto",
                   choices=["auto", "replicated", "hot-shard", "feature-shard", "shard"],
                   help="auto = replicated at N = 1, hot-shard at N > 1")
    p.add_argument("--hot-frac", type=float, default=0.5,
                   help="hot-shard: share of nodes (highest in-degree) cached on every GPU")
    p.add_argument("--shard", action="store_true", help="alias of --mode shard")
    p.add_argument("--bias", action="store_true",
                   help="biased (degree-weighted) sampler: probs[e] = 1 + indeg(indices[e])")
    p.add_argument("--cache-frac", type=float, default=1.0,
                   help="cache only the ceil(f*N) highest in-degree nodes in HBM; every other "
                        "row is read zero-copy from pinned host memory (SURVEY 8(f) rank 2)")
    p.add_argument("--comm", choices=["auto", "gloo", "rccl"], default="auto",
                   help="transport of the library's setup collectives at N > 1 (auto: RCCL, "
                        "or the gloo host transport when ranks share a GPU)")
    p.add_argument("--depth", type=int, default=3,
                   help="batches in flight (PrefetchLoader streams); 1 = the sequential loop")
    p.add_argument("--no-replicated-pass", action="store_true",
                   help="N > 1: skip the secondary replicated measurement")
    p.add_argument("--no-xgmi-pass", action="store_true",
                   help="N > 1: skip the secondary feature-shard (xGMI gather) measurement")
    p.add_argument("--check-batches", type=int, default=4,
                   help="N > 1: batches of the pre-timing self-check (0 = no check)")
    p.add_argument("--seq-calls", type=int, default=50,
                   help="synchronous calls timed for sequential_value (SURVEY 8(d): >= 50)")
    p.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--seed", type=int, default=20261015)
    p.add_argument("--setup-timeout", type=float, default=300.0,
                   help="N > 1: bound (s) of every setup / collective phase; a rank stalled "
                        "longer exits non-zero naming the phase (DistGNN.dist.SetupWatchdog)")
    p.add_argument("--secondary", choices=["auto", "none", "papers_bias"], default="auto",
                   help="N = 1: also measure configs[3] (papers100M-like, biased) as a nested "
                        "record (auto: when the primary workload is the default one)")
    a = p.parse_args(argv)
    if a.shard:
        a.mode = "shard"
    return a


def baseline_config(args, mode, hot):
    """The BASELINE.json config this run's workload stands for."""
    if hot is not None:
        return "SURVEY 8(f) rank 2"
    if (args.scale, args.ef) == (27, 12) and args.bias and mode == "replicated":
        return "configs[3] (its graph and sampler, on one GPU)"
    return CONFIG_OF_MODE[mode]


def workload_name(scale, ef):
    return WORKLOADS.get((scale, ef), f"RMAT scale {scale} ef {ef}")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv):
    """`--gpus N` without a torchrun environment: run this script as N ranks (one process per
    GPU) and return their exit status.  Nothing here touches the GPU before the ranks start
    (counting devices does not initialise it on this image)."""
    if os.environ.get("DGS_BENCH_SHARE_DEVICE") != "1" and torch.cuda.device_count() < n:
        raise SystemExit(f"bench.py: --gpus {n} but only {torch.cuda.device_count()} GPUs are "
                         "visible (DGS_BENCH_SHARE_DEVICE=1 rehearses N ranks on one GPU)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd)


def check_world(args, world_env):
    """The rank count must be the one asked for: a mismatch would report a different
    configuration than the caller named."""
    world = int(world_env) if world_env is not None else 1
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch N ranks "
                         "with --gpus N (torchrun --nproc-per-node N ... --gpus N)")
    return world


def resolve_mode(args, world):
    if args.mode != "auto":
        return args.mode
    return "replicated" if world == 1 else "hot-shard"


def cache_lists(mode, N, rank, world, hot, hot_feat=None):
    """(sampler cache nids, feature cache nids) of this rank.  hot: the HBM-cached nodes when
    only part of the graph is cached (--cache-frac), else None; hot_feat: hot-shard's
    replicated hot nodes."""
    def shard(all_ids):
        return all_ids[rank::world] if world > 1 else all_ids
    everything = hot if hot is not None else torch.arange(N)
    if mode == "replicated" or world == 1:
        return everything, everything
    if mode == "hot-shard":
        cold = torch.ones(N, dtype=torch.bool)
        cold[hot_feat] = False
        return everything, torch.cat([hot_feat, shard(torch.nonzero(cold).flatten())])
    if mode == "feature-shard":
        return everything, shard(everything)
    return shard(everything), shard(everything)


# ---------------------------------------------------------------------------- inputs
def build_inputs(args, dev):
    """The synthetic inputs on the host: CSC graph, optional degree-weighted probs, features,
    labels (identical on every rank: fixed seeds)."""
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    indptr_d, indices_d = rmat_csc_torch(args.scale, args.ef, seed=args.seed, device=dev)
    N = indptr_d.numel() - 1
    gen = torch.Generator(device=dev)
    gen.manual_seed(11)
    feats_d = torch.randn(N, args.dim, generator=gen, device=dev)
    labels_d = torch.randint(0, 47, (N,), generator=gen, device=dev)
    out = {"indptr": indptr_d.cpu(), "indices": None, "probs": None}
    if args.bias:  # degree-weighted, probs[e] = float32(1 + indeg(indices[e]))
        indeg = torch.bincount(indices_d, minlength=N)
        out["probs"] = (1 + indeg[indices_d]).to(torch.float32).cpu()
        del indeg
    out["indices"] = indices_d.cpu()
    out["feats"] = feats_d.cpu()
    out["labels"] = labels_d.cpu()
    del indptr_d, indices_d, feats_d, labels_d
    torch.cuda.empty_cache()
    return out


def shared_inputs(args, dev, dist, local_rank, tag):
    """N > 1: local rank 0 builds the inputs and writes them to /dev/shm; every rank maps the
    same pages (one host copy per node, as the reference's mp.spawn shares one).  Falls back to
    a copy per rank when /dev/shm cannot hold them (reported in the line)."""
    names = ("indptr", "indices", "probs", "feats", "labels")
    base = f"/dev/shm/dgs_bench_{tag}"
    meta = [None]
    if local_rank == 0:
        inp = build_inputs(args, dev)
        need = sum(t.numel() * t.element_size() for t in inp.values() if t is not None)
        try:
            st = os.statvfs("/dev/shm")
            room = st.f_bavail * st.f_frsize
        except OSError:
            room = 0
        if room > need * 1.05 + (1 << 30):
            m = {}
            for k in names:
                t = inp[k]
                if t is None:
                    continue
                t.numpy().tofile(f"{base}_{k}")
                m[k] = (list(t.shape), str(t.dtype).replace("torch.", ""))
            meta = [m]
        else:
            meta = [{"_local": True}]
    dist.broadcast_object_list(meta, 0)
    m = meta[0]
    if m.get("_local"):
        inp = inp if local_rank == 0 else build_inputs(args, dev)
        dist.barrier()
        return inp, "per-rank copies (/dev/shm too small for one shared copy)"
    out = {"probs": None}
    for k, (shape, dt) in m.items():
        n = int(np.prod(shape))
        out[k] = torch.from_file(f"{base}_{k}", shared=True, size=n,
                                 dtype=getattr(torch, dt)).view(*shape)
    dist.barrier()  # every rank has mapped them: the names can go, the pages stay mapped
    if local_rank == 0:
        for k in m:
            os.unlink(f"{base}_{k}")
    return out, "one copy per node, mapped by every rank from /dev/shm"


def hot_set(indices, N, frac, dev):
    """The ceil(f*N) highest in-degree nodes (ties by id), or None for the whole graph."""
    if frac >= 1.0:
        return None
    n_hot = max(1, int(math.ceil(frac * N)))
    indeg = torch.bincount(indices.to(dev), minlength=N)
    return torch.sort(indeg, descending=True, stable=True).indices[:n_hot].cpu()


def verify_setup(sampler, server, indices, feats, s_cache, f_cache, N, dev):
    """The HBM copies the services made from the host inputs (uploaded through the library's
    pinned staging, or read through pinned host pages) equal the inputs as torch copies them:
    the sampler's cached
    neighbour ids (when it caches every row in id order) and the feature server's cached rows.
    A mismatch ends the run before anything is timed."""
    _, sub_indices, _ = sampler._CAPI_get_local_cache_structure_tensors()
    if s_cache.numel() == N and torch.equal(s_cache, torch.arange(N)):
        want = indices.to(dev)
        bad = int((sub_indices != want).sum()) if sub_indices.numel() == want.numel() else -1
        if bad:
            raise SystemExit(f"bench.py: the sampler's HBM copy of the graph differs from the "
                             f"host graph at {bad} of {want.numel()} neighbour ids")
        del want
    gpu_feat = server._CAPI_get_gpu_feature()
    if gpu_feat is not None and f_cache.numel():
        rows = 0
        for part in torch.split(f_cache, 1 << 20):  # bounded temporaries
            want = feats[part].to(dev)
            got = gpu_feat[rows: rows + part.numel()]
            if not torch.equal(got, want):
                raise SystemExit("bench.py: the feature server's HBM cache differs from the host "
                                 f"features in rows {rows}..{rows + part.numel()}")
            rows += part.numel()
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------- timed run
def timed_pass(dgs, sampler, server, labels_dev, fan_out, args, next_seeds, dist, profile):
    """W warm-up batches, then exactly K timed batches between barrier + synchronize on both
    sides.  Returns (elapsed s, edges, rows, profile dict or None, host step gaps, mallocs)."""
    from DistGNN.dataloading import PrefetchLoader
    dev = labels_dev.device

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

    # Python's cyclic garbage collector is held off from here to the end of the timed region: a
    # full collection over torch's object graph stalls the host for milliseconds (a 10 ms step
    # gap was seen in a 1000-step run), which a 20-step run cannot absorb.  It runs once before
    # the warm-up, not just before t0: a collection walks every Python object and leaves the
    # host's caches cold, and the first timed submissions then took 250 us instead of 70 us
    # (round 5, profiles/r05_bench_gc_placement.txt: 20-step value 2.39-2.48 -> 2.72-2.75 G).
    # No GPU work depends on it.
    gc.collect()
    gc.disable()
    for _ in batches_of([next_seeds() for _ in range(args.warmup)]):
        pass
    _ = None  # (the last warm-up batch is not held into the timed region)
    # the timed batches' seeds (views of the shuffled train set, as SeedGenerator yields them)
    timed = [next_seeds() for _ in range(args.steps)]
    it = batches_of(timed)  # worker threads start here; no batch is submitted before t0
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    # only the gather kernel is measured in the timed region: its workgroups stamp their own
    # start / end (no stream markers between the measured kernels)
    if profile:
        dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    # DGS_BENCH_ALLOC_TRACE=1 (diagnostics): the Python stack of every segment the caching
    # allocator maps inside the timed region, to stderr
    trace = os.environ.get("DGS_BENCH_ALLOC_TRACE") == "1"
    if trace:
        torch.cuda.memory._record_memory_history(max_entries=100000)
    pools = ("segment.large_pool.allocated", "segment.small_pool.allocated")
    st0 = torch.cuda.memory_stats(dev)
    seg0 = [st0.get(k, 0) for k in pools]
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
    gc.enable()
    prof = dgs.ops.profile_read() if profile else None
    # hipMalloc calls the caching allocator made inside the timed region (host stalls)
    st1 = torch.cuda.memory_stats(dev)
    if trace:
        snap = torch.cuda.memory._snapshot()
        torch.cuda.memory._record_memory_history(enabled=None)
        for dt in snap.get("device_traces", []):
            for ev in dt:
                if ev.get("action") == "segment_alloc":
                    frames = [f"{f['filename']}:{f['line']} {f['name']}"
                              for f in ev.get("frames", []) if f.get("filename", "").endswith(".py")]
                    print(f"[bench] segment_alloc {ev.get('size')} B stream {ev.get('stream')}: "
                          + " <- ".join(frames[:6]), file=sys.stderr)
    mallocs = {"large_pool": st1.get(pools[0], 0) - seg0[0],
               "small_pool": st1.get(pools[1], 0) - seg0[1]}
    # host-side spacing of consecutive batches handed out by the loader (jitter diagnostics)
    gaps = np.diff(np.array([t0] + step_t)) * 1e3
    tr = getattr(it, "trace", None)
    if tr:  # DGS_PREFETCH_TRACE=1: the first steps' phases, us after t0
        print("[bench] loader trace: " + " ".join(f"{n}@{(t - t0) * 1e6:.0f}" for n, t in tr),
              file=sys.stderr)
    step_gaps = {"p10": float(np.percentile(gaps, 10)), "p50": float(np.median(gaps)),
                 "p90": float(np.percentile(gaps, 90)), "max": float(gaps.max())}
    return elapsed, edges, rows, prof, step_gaps, mallocs


def reduce_over_ranks(dist, dev, elapsed, *work):
    """Job time = max over ranks (every rank ran the same K steps between barriers); work =
    sum over ranks.  dist is None for a single process."""
    if dist is None:
        return (elapsed,) + tuple(float(w) for w in work)
    t = torch.tensor([elapsed] + [float(w) for w in work], dtype=torch.float64, device=dev)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return (float(mx[0]),) + tuple(float(x) for x in t[1:])


def seed_slice(train, rank, world):
    """Train nids of this rank (node_classification.py:312-321: contiguous equal slices)."""
    per = (train.numel() + world - 1) // world
    return train[rank * per:(rank + 1) * per]


# ---------------------------------------------------------------------------- main
def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = check_world(args, world_env)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    mode = resolve_mode(args, world)
    # DGS_BENCH_SHARE_DEVICE=1 rehearses the N > 1 flow on a 1-GPU box: every rank on cuda:0,
    # gloo process group and host transport (RCCL refuses two ranks on one device).
    share = os.environ.get("DGS_BENCH_SHARE_DEVICE") == "1"
    dev_index = 0 if share else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist = None
    comm = None
    wd = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        from DistGNN.dist.watchdog import SetupWatchdog
        # Bounded failure (round 6): a rank stalled in a collective -- rendezvous, the RCCL
        # communicator, the services' IPC exchange, the self-check, the barriers around the
        # timed region -- ends every rank non-zero within --setup-timeout s per phase, naming
        # the phase, instead of holding the node until an outer limit.
        wd = SetupWatchdog(args.setup_timeout, rank=rank, what="bench")
        wd.step("init_process_group")
        tmo = datetime.timedelta(seconds=args.setup_timeout)
        if share:
            dist.init_process_group("gloo", timeout=tmo)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=tmo)
    import dgs
    if world > 1:
        # the library's setup collectives (IPC handles, cache lists, barriers); none in the
        # timed loop.  Every mode sets it up, so the secondary replicated pass is collective too.
        comm = args.comm if args.comm != "auto" else ("gloo" if share else "rccl")
        wd.step(f"library communicator ({comm})")
        if comm == "rccl":
            if share:
                raise SystemExit("bench.py: RCCL refuses two ranks on one GPU; use --comm gloo")
            from DistGNN.dist import create_communicator
            create_communicator(world)
        else:
            dgs.ops._CAPI_set_host_comm(dist.group.WORLD if share
                                        else dist.new_group(backend="gloo"))

    out = run_workload(args, dgs, dist, world, rank, local_rank, mode, share, dev_index, dev, comm,
                       wd)
    sec = secondary_workload(args, world)
    if sec is not None:
        # configs[3] (papers100M-like graph, degree-weighted biased [15,10,5], d = 128) in the
        # same run: the north star's own sampler config, on one GPU
        a2 = parse(sys.argv[1:])
        for k, v in sec.items():
            setattr(a2, k, v)
        t_sec = time.time()
        try:
            rec = run_workload(a2, dgs, dist, world, rank, local_rank, "replicated", share,
                               dev_index, dev, comm)
            rec["wall_s"] = time.time() - t_sec
        except (RuntimeError, MemoryError, torch.OutOfMemoryError) as e:  # reported, not fatal
            rec = {"skipped": f"{type(e).__name__}: {e}"[:400]}
            torch.cuda.empty_cache()
        out["secondary"] = {"papers_bias": rec}
    if rank == 0:
        print(json.dumps(out), flush=True)
    torch.cuda.synchronize()
    if dist:
        wd.step("final barrier")
        dist.barrier()
        dist.destroy_process_group()
        wd.done()


def secondary_workload(args, world):
    """--secondary auto: the N = 1 default run (products-like uniform, configs[1]) also measures
    configs[3]'s sampler -- papers100M-like RMAT scale 27 x ef 12 (134 M nodes, 1.61 B edges),
    degree-weighted biased [15,10,5], d = 128 -- as a nested record of the same JSON line, with
    the same steps / warm-up and a shorter CPU baseline.  Returns the argument overrides, or
    None."""
    if args.secondary == "none" or world != 1:
        return None
    default = (args.scale, args.ef, args.dim, args.bias, args.cache_frac) == (21, 59, 100, False,
                                                                              1.0)
    if args.secondary == "auto" and not default:
        return None
    return {"scale": 27, "ef": 12, "dim": 128, "bias": True, "mode": "replicated",
            "seq_calls": min(args.seq_calls, 20),
            "cpu_baseline_seconds": min(args.cpu_baseline_seconds, 8.0), "secondary": "none"}


def run_workload(args, dgs, dist, world, rank, local_rank, mode, share, dev_index, dev, comm,
                 wd=None):
    """One workload's bench record: inputs, services, self-check (N > 1), the timed pass, side
    passes and the CPU baseline; the services and inputs are freed before returning.  wd: the
    N > 1 SetupWatchdog, told which phase this rank is in."""
    fan_out = [int(x) for x in args.fan_out.split(",")]

    def phase(name):
        if wd is not None:
            wd.step(name)

    # ---------------- synthetic inputs (identical on every rank)
    t0 = time.time()
    phase("inputs")
    if world > 1:
        port = os.environ.get("MASTER_PORT", "0")
        inp, host_copy = shared_inputs(args, dev, dist, local_rank,
                                       f"{port}_{os.environ.get('TORCHELASTIC_RUN_ID', '')}")
    else:
        inp, host_copy = build_inputs(args, dev), "single process"
    indptr, indices, feats, labels = inp["indptr"], inp["indices"], inp["feats"], inp["labels"]
    probs = inp["probs"] if args.bias else torch.Tensor()
    N = indptr.numel() - 1
    E = indices.numel()
    hot = hot_set(indices, N, args.cache_frac, dev)
    if mode == "hot-shard" and hot is not None:
        raise SystemExit("bench.py: --mode hot-shard caches every row somewhere; it does not "
                         "combine with --cache-frac")
    hot_feat = hot_set(indices, N, args.hot_frac, dev) if mode == "hot-shard" else None
    g2 = torch.Generator()
    g2.manual_seed(2)
    train = torch.randperm(N, generator=g2)[: N // 10]
    train_local = seed_slice(train, rank, world).to(dev)
    log(f"[bench] graph N={N} E={E} d={args.dim} built in {time.time() - t0:.1f}s "
        f"({host_copy})")

    # ---------------- services
    s_cache, f_cache = cache_lists(mode, N, rank, world, hot, hot_feat)
    # the rows this GPU holds (the others come from a peer or the host)
    local_mask = torch.zeros(N, dtype=torch.bool, device=dev)
    local_mask[f_cache.to(dev)] = True
    # which nodes any GPU holds (the rest are host rows), for the host-row share reported below
    cached_mask = torch.zeros(N, dtype=torch.bool, device=dev)
    cached_mask[(hot if hot is not None else torch.arange(N)).to(dev)] = True
    t0 = time.time()
    phase("services (cache build, IPC handle exchange)")
    # A partial cache reads its uncached rows from host memory: the host arrays are pinned in
    # place first, as the reference example pins its graph (node_classification.py:186), so the
    # services read them zero-copy instead of keeping pinned copies of their own.
    pinned = []
    if hot is not None:
        for t in (indptr, indices, probs, feats):
            if t is not None and t.numel() > 0:
                dgs.ops._CAPI_tensor_pin_memory(t)
                pinned.append(t)
    sampler = dgs.classes.P2PCacheSampler(indptr, indices, probs, s_cache, dev_index)
    server = dgs.classes.P2PCacheFeatureServer(feats, f_cache, dev_index)
    labels_dev = labels.to(dev)
    layout = server._layout()
    torch.cuda.synchronize()
    log(f"[bench] services ready in {time.time() - t0:.1f}s (mode {mode})")
    verify_setup(sampler, server, indices, feats, s_cache, f_cache, N, dev)
    # N > 1: the replicated services (whole graph + features in this GPU's HBM) are the
    # self-check's reference and the secondary `replicated` pass (collective constructors:
    # every rank builds them in the same order)
    everything = hot if hot is not None else torch.arange(N)
    ref = None
    # built only when something uses them (a graph that fits one GPU's HBM only when sharded
    # runs with --no-replicated-pass --check-batches 0: the self-check then compares against
    # this layout's own sequential loop, and the xGMI pass samples with this layout's sampler)
    need_ref = not args.no_replicated_pass or args.check_batches > 0
    if world > 1 and mode != "replicated" and need_ref:
        phase("replicated reference services")
        ref = (dgs.classes.P2PCacheSampler(indptr, indices, probs, everything, dev_index),
               dgs.classes.P2PCacheFeatureServer(feats, everything, dev_index))
    self_check = None
    if world > 1:
        phase("multi-rank self-check")
        self_check = multi_rank_self_check(dgs, dist, sampler, server, ref, labels_dev, fan_out,
                                           args, next_seeds_factory(train_local, args), rank,
                                           world, dev, share)
    dgs.ops._CAPI_set_random_seed(args.seed + rank)

    torch.manual_seed(1)
    next_seeds = next_seeds_factory(train_local, args)

    phase("timed pass and side passes")
    elapsed, edges, rows, prof, step_gaps, mallocs = timed_pass(
        dgs, sampler, server, labels_dev, fan_out, args, next_seeds, dist, profile=True)
    row_bytes = args.dim * 4
    per_row = 2 * row_bytes + 8  # read row + write row + read nid
    gather_bytes = rows * per_row
    red_dev = torch.device("cpu") if share else dev
    elapsed_all, edges_all, rows_all, gbytes_all = reduce_over_ranks(
        dist, red_dev, elapsed, edges, rows, gather_bytes)

    side = side_pass(dgs, sampler, server, labels_dev, fan_out, args, next_seeds, cached_mask,
                     local_mask, per_row)

    # roofline of the dominant HBM kernel (feature gather), timed live by its own workgroups
    g_ms = prof["gather_ms"] / max(prof["gather_launches"], 1)
    g_bytes = gather_bytes / max(prof["gather_launches"], 1)
    achieved = g_bytes / (g_ms * 1e-3) / 1e9 if g_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic(args.dim, rows / max(prof["gather_launches"], 1))

    # ---------------- N > 1: the same K steps with everything replicated (secondary figure)
    replicated = None
    if ref is not None and not args.no_replicated_pass:
        dgs.ops._CAPI_set_random_seed(args.seed + rank)
        r_el, r_ed, _, _, _, _ = timed_pass(dgs, ref[0], ref[1], labels_dev, fan_out, args,
                                            next_seeds, dist, profile=False)
        r_el, r_ed = reduce_over_ranks(dist, red_dev, r_el, r_ed)
        replicated = {"value": r_ed / r_el, "unit": "sampled edges/s",
                      "ms_per_step": r_el * 1e3 / args.steps,
                      "workload": "whole graph + features in every GPU's HBM (configs[1] "
                                  "layout on every rank)"}

    # ---------------- N > 1: configs[4]'s xGMI gather -- every feature row sharded v mod N
    xgmi = None
    if world > 1 and mode not in ("feature-shard", "shard") and not args.no_xgmi_pass:
        xgmi = xgmi_pass(dgs, dist, ref[0] if ref is not None else sampler, feats, N, labels_dev,
                         fan_out, args, next_seeds, rank, world, dev_index, red_dev, row_bytes,
                         per_row)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(indptr, indices, inp["probs"] if args.bias else None, feats, train,
                           fan_out, args)

    wl = workload_name(args.scale, args.ef)
    sampler_kind = "biased (degree-weighted)" if args.bias else "uniform"
    if mode == "replicated":
        placement = ("whole graph + features in HBM" +
                     (" on every GPU (independent replicas)" if world > 1 else ""))
    elif mode == "hot-shard":
        placement = (f"graph structure in every GPU's HBM; hot-node feature cache of the "
                     f"{args.hot_frac:.0%} highest in-degree nodes on every GPU, the other rows "
                     f"sharded v mod {world} over the GPUs (P2P feature server, remote rows over "
                     "xGMI)")
    elif mode == "feature-shard":
        placement = (f"graph structure in every GPU's HBM, feature rows sharded v mod {world} "
                     "over the GPUs (P2P feature server, remote rows over xGMI)")
    else:
        placement = (f"graph structure and feature rows sharded v mod {world} over the GPUs "
                     "(remote neighbour lists and rows over xGMI)")
    if hot is not None:
        placement = (f"HBM cache of the {args.cache_frac:.0%} highest in-degree nodes "
                     f"({'replicated' if mode == 'replicated' else 'sharded by rank'}), other "
                     "rows zero-copy from pinned host")
    out = {
        "metric": "sampled edges/sec + feature-gather GB/s, fan-out [15,10,5]",
        "value": edges_all / elapsed_all,
        "unit": "sampled edges/s",
        "value_kind": (f"pipelined: DistGNN.dataloading.PrefetchLoader with {args.depth} batches "
                       "in flight (additive API; --depth 1 = the reference loop); "
                       "sequential_value = SURVEY 8(d)'s single synchronous "
                       "_CAPI_sample_node_classifiction call" if args.depth > 1 else
                       "sequential loop (the reference's three calls per batch)"),
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_all * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (RMAT a,b,c,d=.57,.19,.19,.05; randn f32 features; no OGB offline)",
        "config": {
            "workload": (f"{wl} RMAT scale {args.scale} ef {args.ef} (N={N}, E={E}), "
                         f"{sampler_kind} sampler fan-out {fan_out} without replacement, "
                         f"B={args.batch} seeds/step/GPU, + feature gather d={args.dim} f32 + "
                         f"label gather; {placement}"),
            "baseline_config": baseline_config(args, mode, hot),
            "mode": mode,
            "fan_out": fan_out, "batch_per_gpu": args.batch, "num_nodes": N, "num_edges": E,
            "feat_dim": args.dim, "parallelism": f"dp{world} (seed-parallel)",
            "cache_frac": args.cache_frac,
            "pipeline_depth": args.depth,
            "setup_comm": comm,
            "host_graph": host_copy,
            "host_arrays": ("pinned in place (_CAPI_tensor_pin_memory), read zero-copy"
                            if hot is not None else
                            "uploaded once for the cache build (every row cached in HBM)"),
        },
        "sequential_value": side["sequential_value"],
        "sequential_call_ms_median": side["seq_ms_median"],
        "replicated": replicated,
        # N > 1: configs[4]'s gather + xGMI p2p layout (feature rows sharded v mod N, (N-1)/N of
        # the gathered rows read from peers over xGMI), same sampler and batches
        "xgmi_feature_shard": xgmi,
        # N > 1: RCCL / host-transport all-gather of rank-dependent payloads and the first
        # batches of this layout bit-exact against the replicated services (checked before the
        # timed region; a mismatch ends the run non-zero on every rank)
        "self_check": self_check,
        "host_step_gap_ms": step_gaps,
        "python_gc_in_timed_region": ("disabled (gc.collect() before the warm-up, gc.enable() "
                                      "after the timed region)"),
        "allocator_mallocs_in_timed_region": mallocs,
        "host_row_share": side["host_rows"],
        # gathered rows that cached on another GPU (read over xGMI)
        "remote_row_share": side["remote_rows"],
        # host rows cross PCIe Gen5 x16 (63 GB/s spec): their read rate during the gather
        "gather_host_read_GBps": (side["host_rows"] * rows * row_bytes /
                                  (prof["gather_ms"] * 1e-3) / 1e9
                                  if prof["gather_ms"] > 0 else 0.0),
        "gather_GBps": achieved,
        "gather_GBps_wall": gbytes_all / elapsed_all / 1e9,
        "gather_GBps_sync_call": side["call_gbps"],
        "sampled_edges_per_step": edges_all / args.steps,
        "gathered_rows_per_step": rows_all / args.steps,
        "gather_kernel_ms_per_step": prof["gather_ms"] / args.steps,
        "sample_span_ms_per_call": side["sample_span_ms"],
        "label_select_kernel_ms": side["select_ms"],
        # the whole step against the floors of all its kernels (HBM bytes + Philox work)
        "step_roofline": step_floor(side.pop("blocks", None), indptr, fan_out, args.bias,
                                    args.dim, elapsed_all * 1e3 / args.steps),
        "roofline": {
            "bound": ("hbm" if world == 1 or mode == "replicated"
                      else "hbm (local rows) + xGMI (remote rows)"),
            "kernel": ("k_gather<16, U, StridedSrc> (P2PCacheFeatureServer gather, computed row "
                       "addresses)" if layout >= 0 else
                       "k_gather<16, U, TableSrc> (P2PCacheFeatureServer gather, address table)") +
                      "; U = 16-B chunks per lane: 8 for launches of >= 2^21 chunks, else 4",
            "timing": ("device-side s_memrealtime stamps per workgroup (first workgroup start to "
                       "last workgroup end of each launch, 100 MHz wall clock) over the timed "
                       "region, where each gather shares the GPU with the sampling kernels of the "
                       "other batches in flight"),
            "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBPS,
            "bytes_per_launch": g_bytes, "avg_launch_ms": g_ms,
            "traffic": traffic,
            "traffic_source": traffic_src,
        },
        # the same gather kernel with nothing running beside it (sequential side pass)
        "roofline_isolated": {
            "achieved": side["iso_gbps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": side["iso_gbps"] / HBM_PEAK_GBPS,
            "avg_launch_ms": side["iso_ms"],
        },
        # SURVEY 8(d)'s gather micro-bench (2^20 random nids, the same feature server)
        "roofline_microbench": {
            "rows": 1 << 20, "nids": "randint(0, N, 2^20), generator seed 3",
            "achieved": side["mb_gbps"], "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": side["mb_gbps"] / HBM_PEAK_GBPS,
            "avg_launch_ms": side["mb_ms"],
        },
        "cpu_baseline": cpu,
    }
    if world > 1 and mode != "replicated":
        # (W-1)/W of a v mod W sharded gather's rows are remote, spread over W-1
        # links of XGMI_LINK_GBPS, so row reads are bounded by W * XGMI_LINK_GBPS per GPU;
        # the algorithmic bytes count each row twice (read + local write)
        out["roofline"]["xgmi_bound_GBps"] = 2 * world * XGMI_LINK_GBPS
        out["roofline"]["frac_of_xgmi_bound"] = (None if share else
                                                 achieved / (2 * world * XGMI_LINK_GBPS))
    # collective destructors (same order on every rank) before the next workload / teardown
    del ref
    del sampler, server
    for t in pinned:
        dgs.ops._CAPI_tensor_unpin_memory(t)
    del pinned
    del inp, indptr, indices, feats, labels, probs, labels_dev, local_mask, cached_mask
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    return out


def next_seeds_factory(train_local, args):
    """Endless SeedGenerator batches of this rank's train nids (shuffled, drop_last)."""
    from DistGNN.dataloading import SeedGenerator
    state = {"it": iter(SeedGenerator(train_local, args.batch, shuffle=True, drop_last=True))}

    def next_seeds():
        try:
            return next(state["it"])
        except StopIteration:
            state["it"] = iter(SeedGenerator(train_local, args.batch, shuffle=True,
                                             drop_last=True))
            return next(state["it"])
    return next_seeds


def check_allgather(dgs, rank, world, dev):
    """_Test_NCCLTensorAllGather (nccl_context.cc:52-112, the library's setup all-gather) with
    rank-dependent lengths, as /root/reference/tests/test_nccl.py:14-21 does: rank r sends
    3 + 5r int64 values r * 1000 + i; every rank checks every payload."""
    mine = torch.arange(3 + 5 * rank, dtype=torch.int64, device=dev) + rank * 1000
    got = dgs.ops._Test_NCCLTensorAllGather(mine)
    if mine.is_cuda:
        torch.cuda.synchronize()
    bad = 0
    for r in range(world):
        want = torch.arange(3 + 5 * r, dtype=torch.int64) + r * 1000
        bad += int(len(got) != world or not torch.equal(got[r].cpu(), want))
    return bad


def compare_batches(got, exp):
    """Mismatching tensors between two lists of (blocks, x, y) batches (bit-exact)."""
    bad = 0
    for (gb, gx, gy), (eb, ex, ey) in zip(got, exp):
        bad += int(len(gb) != len(eb))
        for tg, te in zip(gb, eb):
            bad += sum(int(u.dtype != v.dtype or not torch.equal(u, v)) for u, v in zip(tg, te))
        bad += int(not torch.equal(gx, ex)) + int(not torch.equal(gy, ey))
    return bad + abs(len(got) - len(exp))


def multi_rank_self_check(dgs, dist, sampler, server, ref, labels_dev, fan_out, args,
                          next_seeds, rank, world, dev, share):
    """Before the timed region at N > 1: (a) the setup all-gather with rank-dependent payloads;
    (b) --check-batches batches through this layout's services and PrefetchLoader, bit-exact
    against the replicated services' sequential loop with the same launch seeds (the P2P
    sampler and the peer-row gather draw the same RNG coordinates and copy the same rows,
    rowwise_sampling_p2p.cu:38-39 = rowwise_sampling.cu:62-63).  A failure on any rank ends
    every rank non-zero."""
    from DistGNN.dataloading import PrefetchLoader
    ag_bad = check_allgather(dgs, rank, world, dev)
    batch_bad, n_check = 0, max(0, args.check_batches)
    if n_check:
        seeds = [next_seeds() for _ in range(n_check)]
        rs, rf = ref if ref is not None else (sampler, server)
        dgs.ops._CAPI_set_random_seed(4242 + rank)
        exp = []
        for sd in seeds:
            blocks = rs._CAPI_sample_node_classifiction(sd, fan_out, False)
            exp.append((blocks, rf._CAPI_get_feature(blocks[-1][1]),
                        dgs.ops._CAPI_cuda_index_select(labels_dev, sd)))
        dgs.ops._CAPI_set_random_seed(4242 + rank)
        got = list(PrefetchLoader(sampler, seeds, fan_out, server=server, labels=labels_dev,
                                  depth=args.depth))
        torch.cuda.synchronize()
        batch_bad = compare_batches(got, exp)
        del got, exp
    red = torch.device("cpu") if share else dev
    t = torch.tensor([ag_bad, batch_bad], dtype=torch.int64, device=red)
    dist.all_reduce(t)
    ag_all, batch_all = int(t[0]), int(t[1])
    res = {"allgather": "ok" if ag_all == 0 else f"{ag_all} bad payloads",
           "batches_per_rank": n_check, "mismatched_tensors": batch_all,
           "reference": "replicated services, sequential loop" if ref is not None
           else "this layout's sequential loop", "ranks": world}
    if ag_all or batch_all:
        log(f"[bench] multi-rank self-check FAILED: {res}")
        raise SystemExit(1)
    log(f"[bench] multi-rank self-check ok: {res}")
    return res


def xgmi_pass(dgs, dist, sampler, feats, N, labels_dev, fan_out, args, next_seeds, rank, world,
              dev_index, red_dev, row_bytes, per_row):
    """configs[4]'s gather + xGMI p2p layout at N > 1: every feature row sharded v mod N behind
    the P2P feature server (strided addressing, (N-1)/N of the gathered rows read one-sided from
    peers over xGMI), the same K steps.  Checked bit-exact on --check-batches batches against a
    local gather first.  Reports the gather kernel's rate against the xGMI bound."""
    from DistGNN.dataloading import PrefetchLoader
    fs = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(rank, N, world), dev_index)
    dev = labels_dev.device
    bad = 0
    for _ in range(max(1, args.check_batches)):
        blocks = sampler._CAPI_sample_node_classifiction(next_seeds(), fan_out, False)
        nids = blocks[-1][1]
        bad += int(not torch.equal(fs._CAPI_get_feature(nids), feats[nids.cpu()].to(dev)))
    remote = float((blocks[-1][1] % world != rank).double().mean())
    dgs.ops._CAPI_set_random_seed(args.seed + rank)
    el, ed, rows, prof, _, _ = timed_pass(dgs, sampler, fs, labels_dev, fan_out, args, next_seeds,
                                          dist, profile=True)
    g_ms = prof["gather_ms"] / max(prof["gather_launches"], 1)
    achieved = rows * per_row / max(prof["gather_launches"], 1) / (g_ms * 1e-3) / 1e9 \
        if g_ms > 0 else 0.0
    el_all, ed_all, bad_all, ach_all = reduce_over_ranks(dist, red_dev, el, ed, bad, achieved)
    del fs
    torch.cuda.synchronize()
    if bad_all:
        log(f"[bench] xGMI feature-shard gather check FAILED on {int(bad_all)} batches")
        raise SystemExit(1)
    bound = 2 * world * XGMI_LINK_GBPS
    shared = os.environ.get("DGS_BENCH_SHARE_DEVICE") == "1"
    return {"mode": "feature-shard", "value": ed_all / el_all, "unit": "sampled edges/s",
            "ms_per_step": el_all * 1e3 / args.steps, "layout": fs_layout_name(world),
            "remote_row_share": remote, "checked_batches": max(1, args.check_batches),
            "gather_GBps_per_gpu": ach_all / world, "avg_launch_ms": g_ms,
            "xgmi_bound_GBps": bound,
            # ranks sharing one GPU read their "peer" rows from the same HBM: no xGMI bound
            "frac_of_xgmi_bound": None if shared else ach_all / world / bound,
            "ranks_share_one_gpu": shared,
            "frac_of_hbm": ach_all / world / HBM_PEAK_GBPS}


def fs_layout_name(world):
    return (f"feature rows v mod {world} over the GPUs (strided addressing), structure "
            "replicated")


def pmc_traffic(dim, rows_per_launch):
    """HBM bytes per gather launch from the committed PMC calibration of this row size
    (rocprofv3 FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic.py), or None when no
    calibration exists for `dim`: counters cannot be read from inside this process."""
    for name in (f"gather_pmc_d{dim}.json", "gather_pmc.json"):
        path = os.path.join(ROOT, "profiles", name)
        if not os.path.exists(path):
            continue
        try:
            pmc = json.load(open(path))
        except (OSError, ValueError):
            continue
        if pmc.get("dim") == dim and pmc.get("hbm_bytes_per_row"):
            return (pmc["hbm_bytes_per_row"] * rows_per_launch,
                    f"profiles/{name} (rocprofv3 FETCH_SIZE/WRITE_SIZE per row at d={dim}) x "
                    "this run's rows per launch")
    return None, f"no PMC calibration committed for d={dim}"


def side_pass(dgs, sampler, server, labels_dev, fan_out, args, next_seeds, cached_mask,
              local_mask, per_row):
    """Outside the timed region: SURVEY 8(d)'s synchronous per-call figures (median of
    --seq-calls device-synchronised calls after 3 warm-ups), the sample call's GPU span, the
    label select kernel, and the feature gather on its own."""
    n_side = max(args.seq_calls, 3)
    side_seeds = [next_seeds() for _ in range(n_side + 3)]
    torch.cuda.synchronize()
    for s in side_seeds[:3]:
        sampler._CAPI_sample_node_classifiction(s, fan_out, False)
    torch.cuda.synchronize()
    side_nids, rates, call_ms, side_blocks = [], [], [], []
    for s in side_seeds[3:]:
        torch.cuda.synchronize()
        tc = time.perf_counter()
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - tc
        call_ms.append(dt * 1e3)
        rates.append(sum(b[2].numel() for b in blocks) / dt)
        side_nids.append(blocks[-1][1])
        if len(side_blocks) < 8:
            side_blocks.append(blocks)
    # GPU span of a sample call and the label select kernel (profiled, sequential)
    dgs.ops.profile_enable(dgs.ops.PROFILE_SAMPLE | dgs.ops.PROFILE_SELECT)
    for s in side_seeds[3:23]:
        dgs.ops._CAPI_cuda_index_select(labels_dev, s)
        sampler._CAPI_sample_node_classifiction(s, fan_out, False)
    torch.cuda.synchronize()
    sp = dgs.ops.profile_read()
    # share of the gathered rows that are host rows
    host_rows = sum(float((~cached_mask[n.long()]).sum()) / max(n.numel(), 1)
                    for n in side_nids) / max(len(side_nids), 1)
    remote_rows = sum(float((cached_mask[n.long()] & ~local_mask[n.long()]).sum()) /
                      max(n.numel(), 1) for n in side_nids) / max(len(side_nids), 1)
    dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    iso_rows = 0
    for n in side_nids:
        iso_rows += server._CAPI_get_feature(n).shape[0]
    torch.cuda.synchronize()
    iso = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    # SURVEY 8(d) gather micro-bench: n = 2^20 uniform random nids (generator seed 3) through the
    # same feature server, 5 launches after a warm-up, kernel time from the same stamps
    dev = labels_dev.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    mb_nids = torch.randint(0, cached_mask.numel(), (1 << 20,), generator=gen, device=dev)
    server._CAPI_get_feature(mb_nids)
    torch.cuda.synchronize()
    dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    for _ in range(5):
        server._CAPI_get_feature(mb_nids)
    torch.cuda.synchronize()
    mb = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    mb_launches = max(mb["gather_launches"], 1)
    mb_ms = mb["gather_ms"] / mb_launches
    del mb_nids
    # SURVEY 8(d) metric (2): algorithmic bytes / wall time of one synchronous _CAPI_get_feature
    # call (host launch + kernel + synchronisation), median over the side pass
    g_rates = []
    for n in side_nids:
        torch.cuda.synchronize()
        tc = time.perf_counter()
        server._CAPI_get_feature(n)
        torch.cuda.synchronize()
        g_rates.append(n.numel() * per_row / (time.perf_counter() - tc) / 1e9)
    return {
        "blocks": side_blocks,
        "sequential_value": float(np.median(rates)),
        "seq_ms_median": float(np.median(call_ms)),
        "sample_span_ms": sp["sample_ms"] / max(sp["sample_calls"], 1),
        "select_ms": sp["select_ms"] / max(sp["select_launches"], 1),
        "host_rows": host_rows,
        "remote_rows": remote_rows,
        "iso_gbps": (iso_rows * per_row / (iso["gather_ms"] * 1e-3) / 1e9
                     if iso["gather_ms"] > 0 else 0.0),
        "iso_ms": iso["gather_ms"] / max(iso["gather_launches"], 1),
        "call_gbps": float(np.median(g_rates)) if g_rates else 0.0,
        "mb_ms": mb_ms,
        "mb_gbps": (1 << 20) * per_row / (mb_ms * 1e-3) / 1e9 if mb_ms > 0 else 0.0,
    }


# VALU issue floor of the two Philox-bound sampling kernels: wave64 VALU instructions per unit of
# work (uniform hub reservoir: ~30 per 64 draws, SQ counters, profiles/r02_sampling_pmc_sq.txt;
# biased stream: 107 per 512 hub edges -- a 256-edge chunk per half-wave),
# issued at one wave64 instruction per 4 cycles on each of the 1024 SIMDs at 2.4 GHz.  The kernels'
# measured steady-state rates (1.15 T draws/s, 0.72 T hub edges/s) are reported beside it.
PEAK_WAVE_INSTR_PER_S = 1024 * 2.4e9 / 4
UNIFORM_INSTR_PER_DRAW = 30.0 / 64.0
BIAS_INSTR_PER_EDGE = 107.0 / 512.0
UNIFORM_DRAWS_PER_S = 1.15e12
BIAS_EDGES_PER_S = 0.72e12
BIAS_HUB_DEG = 1024     # k_bias_boot / k_bias_stream take rows above this degree
BIAS_BOOT_SAMPLE = 4096


def step_floor(blocks_list, indptr, fan_out, bias, dim, ms_per_step):
    """Step-level roofline (VERDICT r05 "Next round" 7): per batch, the SURVEY 8(d) algorithmic
    HBM bytes of every kernel of the step at 8 TB/s (sampling per hop: 8S seeds + 16S indptr
    pairs + 8 nnz ids + 16 nnz COO + relabel 8(S+nnz) read + 8 S' unique + 16 nnz rewrite, biased
    + 4 sum(deg) probabilities; feature gather 2 d 4 + 8 per row; label gather 24 per seed),
    and the Philox work of the VALU-bound kernels at the VALU issue peak (uniform: one draw per
    reservoir step, sum over rows of deg - k; biased: one draw per edge of every row with
    deg > k, plus the boot's sample of the hub rows).  Averaged over the side pass's batches.
    `sum_us` assumes no overlap between kernels; `max_us` perfect overlap of HBM and VALU work;
    the step can be no faster than max_us.  `valu_at_measured_rate_us`: the same work at the
    kernels' measured steady-state rates."""
    if not blocks_list:
        return None
    ip = indptr.numpy() if hasattr(indptr, "numpy") else indptr
    hbm, valu, meas, draws = [], [], [], []
    for blocks in blocks_list:
        L = len(blocks)
        b_bytes, d = 0.0, 0.0
        for h, (seeds, fr, r, _) in enumerate(blocks):
            k = fan_out[L - 1 - h]
            sd = seeds.cpu().numpy()
            deg = (ip[sd + 1] - ip[sd]).astype(np.float64)
            S, nnz, Sp = sd.size, r.numel(), fr.numel()
            b_bytes += 8 * S + 16 * S + 8 * nnz + 16 * nnz + 8 * (S + nnz) + 8 * Sp + 16 * nnz
            big = deg[deg > k]
            if bias:
                b_bytes += 4 * big.sum()
                d += big.sum() + np.minimum(big[big > BIAS_HUB_DEG], BIAS_BOOT_SAMPLE).sum()
            else:
                d += (big - k).sum()
        rows = blocks[-1][1].numel()
        b_bytes += rows * (2 * dim * 4 + 8) + 24 * blocks[0][0].numel()
        hbm.append(b_bytes)
        draws.append(d)
        valu.append(d * (BIAS_INSTR_PER_EDGE if bias else UNIFORM_INSTR_PER_DRAW) /
                    PEAK_WAVE_INSTR_PER_S)
        meas.append(d / (BIAS_EDGES_PER_S if bias else UNIFORM_DRAWS_PER_S))
    hbm_us = float(np.mean(hbm)) / (HBM_PEAK_GBPS * 1e3)
    valu_us = float(np.mean(valu)) * 1e6
    step_us = ms_per_step * 1e3
    return {
        "hbm_bytes_per_step": float(np.mean(hbm)),
        "hbm_floor_us": hbm_us,
        "philox_draws_per_step": float(np.mean(draws)),
        "valu_floor_us": valu_us,
        "valu_rate": (f"{BIAS_INSTR_PER_EDGE:.3f} wave64 VALU instructions per hub edge "
                      "(k_bias_stream)" if bias else
                      f"{UNIFORM_INSTR_PER_DRAW:.3f} wave64 VALU instructions per draw "
                      "(k_hub_reservoir)") +
                     f" at {PEAK_WAVE_INSTR_PER_S / 1e12:.3f} T wave64 instructions/s",
        "valu_at_measured_rate_us": float(np.mean(meas)) * 1e6,
        "sum_us": hbm_us + valu_us,
        "max_us": max(hbm_us, valu_us),
        "ms_per_step": ms_per_step,
        "frac_of_sum": (hbm_us + valu_us) / step_us if step_us > 0 else 0.0,
        "frac_of_max": max(hbm_us, valu_us) / step_us if step_us > 0 else 0.0,
        "batches": len(blocks_list),
    }


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
    quota = None
    try:  # cgroup v2 CPU quota of this container, in CPUs
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "usable_cpus": usable,
            "cgroup_cpu_quota": quota, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def baseline_threads(info):
    """The per-GPU share of the host: the container's CPU quota when one is set, else the
    usable CPUs over the node's 8 GPUs (DGS_CPU_THREADS overrides).  Returns (threads, why)."""
    if os.environ.get("DGS_CPU_THREADS"):
        return int(os.environ["DGS_CPU_THREADS"]), "DGS_CPU_THREADS"
    if info["cgroup_cpu_quota"]:
        return max(1, int(info["cgroup_cpu_quota"])), "this container's cgroup CPU quota"
    usable = info["usable_cpus"] or os.cpu_count() or 8
    return max(1, usable // 8), "usable CPUs / 8 GPUs per node"


def cpu_baseline(indptr, indices, probs, feats, train, fan_out, args):
    """The oracle's OpenMP restatement on the host cores (DGL is not installed): row-wise
    sampling per hop (uniform, or biased when probs is given) + relabel + feature gather, same
    graph and batch size."""
    from oracle import oracle as O
    info = host_info()
    threads, why = baseline_threads(info)
    ip, ix = indptr.numpy(), indices.numpy()
    pr = probs.numpy() if probs is not None else None
    fx = feats.numpy()
    rng = np.random.default_rng(1)
    seeds_all = train.numpy()
    edges = rows = batches = 0
    t_gather = 0.0
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
        tg = time.perf_counter()
        x = O.index_select(fx, cur, nthreads=threads)
        t_gather += time.perf_counter() - tg
        rows += x.shape[0]
        batches += 1
        if time.perf_counter() - t0 > args.cpu_baseline_seconds:
            break
    dt = time.perf_counter() - t0
    per_row = 2 * args.dim * 4 + 8
    # the CPU gather baseline proper is torch.index_select on the host feature
    # tensor.  Cache-cold: a fresh random id set of the frontier's size for every repeat, over
    # all N rows (the feature matrix is far larger than the last-level cache).
    torch.set_num_threads(threads)
    n_ids = int(cur.size)
    g = torch.Generator().manual_seed(5)
    id_sets = [torch.randint(0, feats.shape[0], (n_ids,), generator=g) for _ in range(16)]
    reps, t1 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t1 < 1.0:
        torch.index_select(feats, 0, id_sets[reps % len(id_sets)])
        reps += 1
    ts_gbps = reps * n_ids * per_row / (time.perf_counter() - t1) / 1e9
    return {"value": edges / dt, "unit": "sampled edges/s", "cores": threads,
            "cores_basis": why, "kind": "port", "host": info,
            "gather_GBps": rows * per_row / t_gather / 1e9 if t_gather > 0 else 0.0,
            "gather_GBps_torch_index_select_cold": ts_gbps,
            "sample": (f"{batches} batches of B={args.batch}, fan-out {fan_out}, same graph; "
                       f"oracle/dgs_oracle.c OpenMP {'biased' if probs is not None else 'uniform'} "
                       f"sampler ({threads} threads) + serial relabel + OpenMP gather, {dt:.1f}s "
                       f"(gather_GBps: the gather's own time, {t_gather:.2f}s)")}


if __name__ == "__main__":
    if os.environ.get("WORLD_SIZE", "1") != "1":
        # a failed rank exits at once: unwinding would wait in teardown collectives for ranks
        # that are themselves waiting for it
        try:
            main()
        except BaseException:
            import traceback
            traceback.print_exc()
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(1)
    else:
        main()
