"""Host cost of the PrefetchLoader per batch (diagnostics): total loop time per batch, the
part spent waiting for a batch's sizes (the GPU), and the rest (Python + C-ABI work).

    python tools/loader_host.py [--batch 1024] [--depth 3] [--steps 2000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402

import dgs  # noqa: E402
from dgs import classes as C  # noqa: E402
from DistGNN.dataloading import PrefetchLoader  # noqa: E402
from DistGNN.dataloading.synthetic import rmat_csc_torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--depth", type=int, default=3)
    p.add_argument("--steps", type=int, default=2000)
    p.add_argument("--scale", type=int, default=21)
    p.add_argument("--ef", type=int, default=59)
    p.add_argument("--fan-out", type=str, default="15,10,5")
    p.add_argument("--dim", type=int, default=100)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix = rmat_csc_torch(a.scale, a.ef, seed=20261015, device=dev)
    N = ip.numel() - 1
    feats = torch.randn(N, a.dim, device=dev).cpu()
    fan_out = [int(x) for x in a.fan_out.split(",")]
    labels = torch.randint(0, 47, (N,), device=dev)
    sampler = C.P2PCacheSampler(ip.cpu(), ix.cpu(), torch.Tensor(), torch.arange(N), 0)
    server = C.P2PCacheFeatureServer(feats, torch.arange(N), 0)
    g = torch.Generator().manual_seed(2)
    train = torch.randperm(N, generator=g)[: N // 10].to(dev)
    batches = [train[(i * a.batch) % (train.numel() - a.batch):][:a.batch]
               for i in range(a.steps)]
    wait = [0.0]
    orig = C._PendingSample.result

    def timed(self, cast=True):
        t = time.perf_counter()
        try:
            return orig(self, cast)
        finally:
            wait[0] += time.perf_counter() - t

    for _ in PrefetchLoader(sampler, batches[:50], fan_out, server=server, labels=labels,
                            depth=a.depth):
        pass
    torch.cuda.synchronize()
    C._PendingSample.result = timed
    t0 = time.perf_counter()
    for _ in PrefetchLoader(sampler, batches, fan_out, server=server, labels=labels,
                            depth=a.depth):
        pass
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    C._PendingSample.result = orig
    n = len(batches)
    print(f"B={a.batch} fan-out {fan_out} depth={a.depth}: {tot / n * 1e6:.1f} us/batch total, "
          f"{wait[0] / n * 1e6:.1f} us waiting for sizes, "
          f"{(tot - wait[0]) / n * 1e6:.1f} us host work")


if __name__ == "__main__":
    main()
