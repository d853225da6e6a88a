"""Biased hub-row statistics of a few synchronous sample calls (run with DGS_BIAS_STATS=1: each
hop prints its hub rows, hub edges, stream chunks and the candidates the stream kernel left for
the merge), then the median span of 20 profiled calls.  bench.py's inputs: RMAT (a,b,c,d =
.57,.19,.19,.05), degree-weighted probs p[e] = 1 + indeg(indices[e]), B = 1024, [15,10,5].

    DGS_BIAS_STATS=1 python tools/r04_bias_stats.py --scale 27 --ef 12
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.environ.get("DGS_BENCH_PYDIR", os.path.join(ROOT, "dist-gnn_amd", "python")))

import torch  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--scale", type=int, default=21)
    p.add_argument("--ef", type=int, default=59)
    p.add_argument("--calls", type=int, default=2)
    a = p.parse_args()
    import dgs
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr, indices = rmat_csc_torch(a.scale, a.ef, seed=20261015, device=dev)
    N = indptr.numel() - 1
    indeg = torch.bincount(indices, minlength=N)
    probs = (1 + indeg[indices]).to(torch.float32).cpu()
    del indeg
    sampler = dgs.classes.P2PCacheSampler(indptr.cpu(), indices.cpu(), probs, torch.arange(N), 0)
    del indptr, indices
    torch.cuda.empty_cache()
    g = torch.Generator(device=dev).manual_seed(2)
    dgs.ops._CAPI_set_random_seed(20261015)
    for _ in range(a.calls):
        s = torch.randint(0, N, (1024,), generator=g, device=dev)
        blocks = sampler._CAPI_sample_node_classifiction(s, [15, 10, 5], False)
        torch.cuda.synchronize()
        print("edges", sum(b[2].numel() for b in blocks), flush=True)
    os.environ.pop("DGS_BIAS_STATS", None)


if __name__ == "__main__":
    main()
