"""cProfile of the PrefetchLoader loop on the arxiv-like (host-bound) shape: where the
per-batch Python time goes (diagnostics).   python tools/loader_pyprof.py [--steps 3000]"""
import argparse
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))

import torch  # noqa: E402

import dgs  # noqa: E402
from DistGNN.dataloading import PrefetchLoader  # noqa: E402
from DistGNN.dataloading.synthetic import rmat_csc_torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=3000)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    indptr, indices = rmat_csc_torch(17, 9, seed=1, device=dev)
    N = indptr.numel() - 1
    feats = torch.randn(N, 128)
    labels = torch.randint(0, 40, (N,), device=dev)
    sampler = dgs.classes.P2PCacheSampler(indptr.cpu(), indices.cpu(), torch.Tensor(),
                                          torch.arange(N), 0)
    server = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(N), 0)
    g = torch.Generator().manual_seed(0)
    batches = [torch.randint(0, N, (1024,), generator=g).to(dev) for _ in range(a.steps)]
    for _ in PrefetchLoader(sampler, batches[:50], [10, 10], server=server, labels=labels, depth=3):
        pass
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in PrefetchLoader(sampler, batches, [10, 10], server=server, labels=labels, depth=3):
        pass
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
