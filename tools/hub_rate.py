"""Draw rate of the uniform hub-reservoir kernel per hop (diagnostics).

Runs sequential sample calls on the products-like bench graph and counts, per hop, the
reservoir draws of the hub rows (rows with deg - k > 128: sum of deg - k); run it under
rocprofv3 --kernel-trace and pass the trace to --trace to get draws/s per hub launch:

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/hubrate -- \
        python3 tools/hub_rate.py --calls 20 --out gpurun_out/hub_draws.json
    python3 tools/hub_rate.py --report gpurun_out/hub_draws.json --trace <kernel_trace.csv>
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dist-gnn_amd", "python"))


def run(args):
    import torch
    import dgs
    from DistGNN.dataloading.synthetic import rmat_csc_torch
    dev = torch.device("cuda", 0)
    indptr_d, indices_d = rmat_csc_torch(args.scale, args.ef, seed=20261015, device=dev)
    deg = (indptr_d[1:] - indptr_d[:-1])
    N = deg.numel()
    probs = torch.Tensor()
    if args.bias:  # bench.py --bias: degree-weighted
        indeg = torch.bincount(indices_d, minlength=N)
        probs = (1 + indeg[indices_d]).to(torch.float32).cpu()
        del indeg
    sampler = dgs.classes.P2PCacheSampler(indptr_d.cpu(), indices_d.cpu(), probs,
                                          torch.arange(N), 0)
    fan_out = [int(x) for x in args.fan_out.split(",")]
    g = torch.Generator().manual_seed(2)
    train = torch.randperm(N, generator=g)[: N // 10]
    dgs.ops._CAPI_set_random_seed(1)
    per_hop = [[] for _ in fan_out]
    for c in range(args.calls):
        s = train[c * args.batch:(c + 1) * args.batch].to(dev)
        blocks = sampler._CAPI_sample_node_classifiction(s, fan_out, False)
        for h, (seeds, _, _, _) in enumerate(blocks):
            k = fan_out[len(fan_out) - 1 - h]
            d = deg[seeds]
            # uniform: reservoir draws of rows with deg - k > 128; biased: every edge of the rows
            # with deg > 1024 (one key each)
            hub = d > 1024 if args.bias else d - k > 128
            draws = int(d[hub].sum()) if args.bias else int((d[hub] - k).sum())
            per_hop[h].append({"draws": draws, "hub_rows": int(hub.sum()),
                               "rows": int(seeds.numel()),
                               "max_deg": int(d.max()) if d.numel() else 0})
    torch.cuda.synchronize()
    json.dump({"fan_out": fan_out, "per_hop": per_hop}, open(args.out, "w"))
    for h, v in enumerate(per_hop):
        print(f"hop {h}: avg draws {sum(x['draws'] for x in v) / len(v):.0f}, "
              f"hub rows {sum(x['hub_rows'] for x in v) / len(v):.0f}, rows "
              f"{sum(x['rows'] for x in v) / len(v):.0f}")


def synthetic(args):
    """One hub row of degree D sampled by `rows` seeds (the same row repeated), one hop: the
    kernel's steady-state draw rate without row switches."""
    import numpy as np
    import torch
    import dgs
    D, rows = args.synthetic_hub, args.rows
    indptr = torch.tensor([0, D], dtype=torch.int64)
    indices = torch.zeros(D, dtype=torch.int64)
    probs = torch.rand(D, generator=torch.Generator().manual_seed(1)) + 0.01 if args.bias \
        else torch.Tensor()
    sampler = dgs.classes.P2PCacheSampler(indptr, indices, probs, torch.arange(1), 0)
    k = int(args.fan_out.split(",")[-1])
    s = torch.zeros(rows, dtype=torch.int64, device="cuda")
    per_hop = [[]]
    for c in range(args.calls):
        sampler._CAPI_sample_node_classifiction(s, [k], False)
        per_hop[0].append({"draws": rows * (D if args.bias else D - k), "hub_rows": rows,
                           "rows": rows,
                           "max_deg": D})
    torch.cuda.synchronize()
    json.dump({"fan_out": [k], "per_hop": per_hop}, open(args.out, "w"))


def report(args):
    d = json.load(open(args.report))
    L = len(d["fan_out"])
    durs = []
    for r in csv.DictReader(open(args.trace)):
        if args.kernel in r["Kernel_Name"]:
            durs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    durs = [x[1] for x in sorted(durs)]
    calls = len(d["per_hop"][0])
    durs = durs[-calls * L:]  # the measured calls are the last ones
    for h in range(L):
        ns = [durs[c * L + h] for c in range(calls)]
        draws = [d["per_hop"][h][c]["draws"] for c in range(calls)]
        rate = sum(draws) / (sum(ns) * 1e-9)
        print(f"hop {h}: avg {sum(ns) / calls / 1e3:.1f} us per launch, "
              f"{sum(draws) / calls / 1e6:.2f} M draws, {rate / 1e9:.0f} G draws/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--calls", type=int, default=20)
    p.add_argument("--batch", type=int, default=1024)
    p.add_argument("--scale", type=int, default=21)
    p.add_argument("--ef", type=int, default=59)
    p.add_argument("--fan-out", default="15,10,5")
    p.add_argument("--out", default="gpurun_out/hub_draws.json")
    p.add_argument("--report")
    p.add_argument("--trace")
    p.add_argument("--synthetic-hub", type=int, default=0)
    p.add_argument("--bias", action="store_true")
    p.add_argument("--kernel", default="k_hub_reservoir",
                   help="kernel whose launches --report prices (k_bias_stream for --bias)")
    p.add_argument("--rows", type=int, default=1)
    a = p.parse_args()
    report(a) if a.report else (synthetic(a) if a.synthetic_hub else run(a))
