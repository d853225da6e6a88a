"""Where one sample call's latency goes: from a rocprofv3 kernel trace of the sequential loop
(bench.py --depth 1), every call's kernels in stream order (a call runs from its hop-0 k_prep to
the kernel before the next k_prep), with each kernel's duration and the idle gap before it,
averaged over the calls by position.

    python tools/call_breakdown.py <kernel_trace.csv> [--skip 10]
"""
import argparse
import csv
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from timeline import short_name  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--skip", type=int, default=10, help="calls to skip (warm-up)")
    a = p.parse_args()
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short_name(r["Kernel_Name"]))
                  for r in csv.DictReader(open(a.trace)))
    # DGS kernels only (torch's own kernels of the bench set-up are dropped)
    rows = [x for x in rows if x[2].startswith("k_")]
    calls, cur = [], None
    for x in rows:
        if x[2] == "k_prep":
            if cur:
                calls.append(cur)
            cur = []
        if cur is not None:
            cur.append(x)
    if cur:
        calls.append(cur)
    calls = calls[a.skip:]
    shape = {}
    for c in calls:
        shape.setdefault(tuple(n for _, _, n in c), []).append(c)
    sig, group = max(shape.items(), key=lambda kv: len(kv[1]))
    print(f"{len(calls)} calls, {len(group)} with the most common kernel sequence "
          f"({len(sig)} kernels)")
    tot_d = tot_g = 0.0
    print(f"{'#':>3} {'kernel':42s} {'gap us':>8} {'dur us':>8} {'end us':>8}")
    for i, name in enumerate(sig):
        d = sum(c[i][1] - c[i][0] for c in group) / len(group) / 1e3
        g = (sum(c[i][0] - c[i - 1][1] for c in group) / len(group) / 1e3) if i else 0.0
        end = sum(c[i][1] - c[0][0] for c in group) / len(group) / 1e3
        tot_d += d
        tot_g += g
        print(f"{i:3d} {name:42s} {g:8.2f} {d:8.2f} {end:8.2f}")
    print(f"    kernels {tot_d:.1f} us + gaps {tot_g:.1f} us")


if __name__ == "__main__":
    main()
