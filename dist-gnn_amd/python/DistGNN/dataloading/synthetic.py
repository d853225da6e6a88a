"""Synthetic graph / feature / seed generators for the DGS benchmarks and tests.

OGB datasets are not available offline, so every measurement runs on seeded synthetic
stand-ins with the shapes of SURVEY.md section 8 (RMAT a,b,c,d = .57,.19,.19,.05; int64 CSC
indptr[N+1] / indices[E]; duplicates and self-loops kept).
"""
import numpy as np
import torch

RMAT_ABCD = (0.57, 0.19, 0.19, 0.05)


def _csc_from_edges_numpy(src, dst, num_nodes):
    order = np.argsort(dst, kind="stable")
    indices = src[order].astype(np.int64)
    counts = np.bincount(dst, minlength=num_nodes)
    indptr = np.zeros(num_nodes + 1, dtype=np.int64)
    np.cumsum(counts, out=indptr[1:])
    return indptr, indices


def rmat_csc_numpy(scale, edge_factor, seed=20261015, abcd=RMAT_ABCD):
    """RMAT graph as int64 CSC (numpy), numpy.random.default_rng(seed)."""
    rng = np.random.default_rng(seed)
    n = 1 << scale
    e = n * edge_factor
    a, b, c, _ = abcd
    src = np.zeros(e, dtype=np.int64)
    dst = np.zeros(e, dtype=np.int64)
    for lvl in range(scale):
        r = rng.random(e)
        bit_src = (r >= a + b).astype(np.int64)          # quadrants c, d -> src bit 1
        bit_dst = (((r >= a) & (r < a + b)) | (r >= a + b + c)).astype(np.int64)  # b, d
        src |= bit_src << lvl
        dst |= bit_dst << lvl
    return _csc_from_edges_numpy(src, dst, n)


def rmat_csc_torch(scale, edge_factor, seed=20261015, device="cuda", abcd=RMAT_ABCD,
                   chunk=1 << 26):
    """RMAT graph as int64 CSC built on `device` with torch's counter-based generator
    (fast for the 100M+ edge benchmark graphs).  Returns (indptr, indices) on `device`."""
    n = 1 << scale
    e = n * edge_factor
    a, b, c, _ = abcd
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    src = torch.empty(e, dtype=torch.int64, device=device)
    dst = torch.empty(e, dtype=torch.int64, device=device)
    for lo in range(0, e, chunk):
        hi = min(e, lo + chunk)
        s = torch.zeros(hi - lo, dtype=torch.int64, device=device)
        d = torch.zeros(hi - lo, dtype=torch.int64, device=device)
        for lvl in range(scale):
            r = torch.rand(hi - lo, generator=gen, device=device)
            s |= (r >= a + b).to(torch.int64) << lvl
            d |= (((r >= a) & (r < a + b)) | (r >= a + b + c)).to(torch.int64) << lvl
        src[lo:hi] = s
        dst[lo:hi] = d
        del s, d
    dst_sorted, order = torch.sort(dst, stable=True)
    indices = src[order]
    del src, order
    counts = torch.bincount(dst_sorted, minlength=n)
    del dst_sorted, dst
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    torch.cumsum(counts, 0, out=indptr[1:])
    return indptr, indices


def degree_probs(indptr, indices):
    """'degree-weighted' edge probabilities: probs[e] = 1 + indeg(indices[e]) (float32)."""
    if isinstance(indptr, torch.Tensor):
        deg = (indptr[1:] - indptr[:-1]).to(torch.float32)
        return 1.0 + deg[indices]
    deg = np.diff(indptr).astype(np.float32)
    return (1.0 + deg[indices]).astype(np.float32)


def parity_features(num_nodes, dim):
    """f[i, j] = float(i*d + j) mod 2^24 -- exactly representable, row-identifying."""
    idx = np.arange(num_nodes * dim, dtype=np.int64) % (1 << 24)
    return idx.astype(np.float32).reshape(num_nodes, dim)
