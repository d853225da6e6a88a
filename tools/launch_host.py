"""Host time of one sample call's launches (diagnostics): the synchronous begin (every hop's
launches issued on the calling thread), the wait for the sizes, and the whole call, each as the
median over many calls of the products-like bench graph.

    python tools/launch_host.py [--batch 1024] [--calls 300]
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

from dgs import classes as C  # noqa: E402
from DistGNN.dataloading.synthetic import rmat_csc_torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--calls", type=int, default=300)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    ip, ix = rmat_csc_torch(21, 59, seed=20261015, device=dev)
    N = ip.numel() - 1
    sampler = C.P2PCacheSampler(ip.cpu(), ix.cpu(), torch.Tensor(), torch.arange(N), 0)
    g = torch.Generator().manual_seed(2)
    train = torch.randperm(N, generator=g)[: N // 10].to(dev)
    fan_out = [15, 10, 5]
    begin, wait, whole = [], [], []
    for i in range(a.calls + 20):
        seeds = train[(i * a.batch) % (train.numel() - a.batch):][:a.batch]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pending = sampler._sample_begin(seeds, fan_out, False, None, host_async=False)
        t1 = time.perf_counter()
        pending.result()
        t2 = time.perf_counter()
        if i >= 20:
            begin.append((t1 - t0) * 1e6)
            wait.append((t2 - t1) * 1e6)
            whole.append((t2 - t0) * 1e6)
    med = statistics.median
    print(f"sample call (B={a.batch}, [15,10,5]): begin (launches on this thread) {med(begin):.1f} us, "
          f"end (wait + views) {med(wait):.1f} us, whole {med(whole):.1f} us")


if __name__ == "__main__":
    main()
