"""Where the synchronous sample call's wall time goes (SURVEY 8(d)'s per-call metric; VERDICT
r05 "Next round" 5), on configs[1] (products-like RMAT scale 21 x 59, uniform [15,10,5],
B = 1024, whole graph in HBM).  The call is timed as bench.py's side pass times it (device
synchronised on both sides), split on the host into: the binding's preparation (_prepare), the
C call (DGS_CALL_TRACE=1 splits it into launches and the wait for the published sizes), the
views, and the closing synchronisation; the GPU span comes from the library's events around
the call (PROFILE_SAMPLE).

    DGS_CALL_TRACE=1 python tools/sync_call_phases.py [--calls 300]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--scale", type=int, default=21)
    ap.add_argument("--ef", type=int, default=59)
    a = ap.parse_args()
    import dgs
    from dgs._lib import c_i64, check, lib, stream_ptr
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    ip, ix = rmat_csc_torch(a.scale, a.ef, device=dev)
    n = ip.numel() - 1
    s = dgs.classes.P2PCacheSampler(ip.cpu(), ix.cpu(), torch.Tensor(), torch.arange(n), 0)
    del ip, ix
    g = torch.Generator()
    g.manual_seed(2)
    train = torch.randperm(n, generator=g)[: n // 10].to(dev)
    fo = [15, 10, 5]
    nb = train.numel() // 1024
    batches = [train[(i % nb) * 1024:(i % nb + 1) * 1024] for i in range(a.calls + 20)]
    for b in batches[:20]:
        s._CAPI_sample_node_classifiction(b, fo, False)
    torch.cuda.synchronize()
    ph = {k: [] for k in ("prepare", "c_call", "views", "sync", "wall")}
    for b in batches[20:]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sd, L, fop, caps, total, buf, _ = s._prepare(b, fo, packed=True)
        t1 = time.perf_counter()
        sizes = (c_i64 * (3 * L))()
        check(lib.dgs_sampler_sample_packed(s._h, sd.data_ptr(), sd.numel(), fop, L, 0,
                                            buf.data_ptr(), sizes, stream_ptr(dev)))
        t2 = time.perf_counter()
        s._views(b, buf, caps, total, sizes, L)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0)):
            ph[k].append(v * 1e6)
    # the same calls through the public entry point (round 6: per-hop views while later hops
    # run), split into the call and the closing synchronisation, and their GPU span
    wall_api, call_api, sync_api = [], [], []
    for b in batches[20:]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s._CAPI_sample_node_classifiction(b, fo, False)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        wall_api.append((t2 - t0) * 1e6)
        call_api.append((t1 - t0) * 1e6)
        sync_api.append((t2 - t1) * 1e6)
    dgs.ops.profile_enable(dgs.ops.PROFILE_SAMPLE)
    for b in batches[20:]:
        s._CAPI_sample_node_classifiction(b, fo, False)
    torch.cuda.synchronize()
    sp = dgs.ops.profile_read()
    dgs.ops.profile_enable(False)
    span = sp["sample_ms"] / max(sp["sample_calls"], 1) * 1e3
    print(f"configs[1]-shaped synchronous calls: {a.calls}, medians in us")
    print("one-call form (dgs_sampler_sample_packed, then all views):")
    for k, v in ph.items():
        print(f"  {k:8s} {np.median(v):8.2f}")
    print("public entry point (_CAPI_sample_node_classifiction):")
    print(f"  call {np.median(call_api):8.2f}  sync {np.median(sync_api):8.2f}")
    print(f"  public entry point wall {np.median(wall_api):8.2f}")
    print(f"  GPU span (events around the call) {span:8.2f}")
    print(f"  outside the span {np.median(wall_api) - span:8.2f}")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
