"""Feature-gather micro-benchmark (nids = randint(0, N, n), n = 2^20 and 2^22,
generator seed 3) through P2PCacheFeatureServer._CAPI_get_feature with every row cached in HBM,
on the three BASELINE feature widths (products d=100, papers d=128, RMAT-1B d=256).

Each launch is timed by the kernel's own workgroup stamps (dgs.ops.profile_*: first workgroup
start to last workgroup end), and the loop is also timed by host wall clock; achieved = the
algorithmic bytes n * (2 * row + 8) over the kernel time.  One JSON line per case on stdout:

    python tools/gather_bench.py > gpurun_out/gather_bench.jsonl
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "dist-gnn_amd", "python"))
import torch  # noqa: E402

import dgs  # noqa: E402

PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
N = 1 << 21          # products-like node count (bench.py --scale 21)
REPS = 20


def run(dim, n):
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    feats = torch.randn(N, dim, generator=gen, device="cuda").cpu()
    server = dgs.classes.P2PCacheFeatureServer(feats, torch.arange(N), 0)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    nids = torch.randint(0, N, (n,), generator=g, device="cuda")
    for _ in range(3):
        out = server._CAPI_get_feature(nids)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), feats[nids.cpu()])  # byte-exact copy
    dgs.ops.profile_enable(dgs.ops.PROFILE_GATHER)
    t0 = time.perf_counter()
    for _ in range(REPS):
        server._CAPI_get_feature(nids)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / REPS
    prof = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    k_ms = prof["gather_ms"] / max(prof["gather_launches"], 1)
    nbytes = n * (2 * dim * 4 + 8)
    achieved = nbytes / (k_ms * 1e-3) / 1e9
    return {"kernel": "k_gather<16, StridedSrc> (P2PCacheFeatureServer, whole graph cached)",
            "num_nodes": N, "dim": dim, "rows": n, "bytes_per_launch": nbytes,
            "avg_launch_us": k_ms * 1e3, "achieved_GBps": achieved, "peak_GBps": PEAK_GBPS,
            "frac": achieved / PEAK_GBPS, "wall_us_per_call": wall * 1e6,
            "wall_GBps": nbytes / wall / 1e9}


def main():
    torch.cuda.set_device(0)
    for dim in (100, 128, 256):
        for n in (1 << 20, 1 << 22):
            print(json.dumps(run(dim, n)), flush=True)


if __name__ == "__main__":
    main()
