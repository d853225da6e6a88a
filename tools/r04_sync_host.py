"""Where the synchronous sample call's wall time goes on the host (SURVEY 8(d)'s metric: one
device-synchronised _CAPI_sample_node_classifiction call).  Products-like graph (bench.py's
configs[1] inputs), B = 1024, [15,10,5]; median over --calls calls of:

  prep   P2PCacheSampler._prepare (dtype checks, plan lookup, output allocation, pointer arrays)
  begin  dgs_sampler_sample_begin: the call's 16 kernel launches on the caller's thread
  end    dgs_sampler_sample_end: the spin until the last scatter publishes the sizes
  views  the per-hop (seeds, frontier, row, col) views
  sync   torch.cuda.synchronize() after the call (the last relabel pass)
  wall   the whole call as bench.py's side pass times it (sync before and after)
plus the GPU span of the call (stream events around its kernels).

    python tools/r04_sync_host.py [--calls 200] [--scale 21 --ef 59]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--calls", type=int, default=200)
    p.add_argument("--scale", type=int, default=21)
    p.add_argument("--ef", type=int, default=59)
    p.add_argument("--batch", type=int, default=1024)
    a = p.parse_args()
    import dgs
    from dgs._lib import c_i64, check, lib
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr, indices = rmat_csc_torch(a.scale, a.ef, seed=20261015, device=dev)
    N = indptr.numel() - 1
    sampler = dgs.classes.P2PCacheSampler(indptr.cpu(), indices.cpu(), torch.Tensor(),
                                          torch.arange(N), 0)
    del indptr, indices
    torch.cuda.empty_cache()
    fan_out = [15, 10, 5]
    g = torch.Generator(device=dev).manual_seed(2)
    seeds = [torch.randint(0, N, (a.batch,), generator=g, device=dev) for _ in range(64)]
    for s in seeds[:5]:
        sampler._CAPI_sample_node_classifiction(s, fan_out, False)
    torch.cuda.synchronize()
    ph = {k: [] for k in ("prep", "begin", "end", "views", "sync", "split_total", "wall")}
    st = dgs._lib.stream_ptr(dev)
    for i in range(a.calls):
        s = seeds[i % len(seeds)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        torch.cuda.synchronize()
        ph["wall"].append(time.perf_counter() - t0)
        # the same call in its pieces
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sv, L, fo, caps, total, buf, ptrs = sampler._prepare(s, fan_out)
        t1 = time.perf_counter()
        check(lib.dgs_sampler_sample_begin(sampler._h, sv.data_ptr(), sv.numel(), fo, L, 0, *ptrs,
                                           None, 0, st))
        t2 = time.perf_counter()
        sizes = (c_i64 * (3 * L))()
        check(lib.dgs_sampler_sample_end(sampler._h, L, sizes, st))
        t3 = time.perf_counter()
        sampler._views(s, buf, caps, total, sizes, L)
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        for k, v in zip(("prep", "begin", "end", "views", "sync", "split_total"),
                        (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t5 - t0)):
            ph[k].append(v)
    dgs.ops.profile_enable(dgs.ops.PROFILE_SAMPLE)
    for i in range(50):
        sampler._CAPI_sample_node_classifiction(seeds[i % len(seeds)], fan_out, False)
        torch.cuda.synchronize()
    span = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    print(f"products-like scale {a.scale} ef {a.ef}, B = {a.batch}, {a.calls} calls, medians (us):")
    for k, v in ph.items():
        print(f"  {k:12s} {statistics.median(v) * 1e6:8.1f}")
    print(f"  gpu span     {span['sample_ms'] / max(span['sample_calls'], 1) * 1e3:8.1f}")


if __name__ == "__main__":
    main()
