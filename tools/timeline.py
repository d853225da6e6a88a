"""GPU occupancy of bench.py's timed region from a rocprofv3 kernel trace: the window runs from
the end of the last warm-up feature gather to the end of the last timed one; reports the
union of kernel intervals (GPU busy), the summed kernel time (concurrency) and the idle gaps.

    python tools/timeline.py <kernel_trace.csv> [--warmup 10] [--steps 100]
"""
import argparse
import csv
import re


def short_name(n):
    """k_name<template args> of a DGS kernel (balanced brackets), else the demangled prefix."""
    m = re.search(r"\bk_\w+", n)
    if not m:
        return n.split("(")[0][:40]
    end, depth = m.end(), 0
    if end < len(n) and n[end] == "<":
        for j in range(end, len(n)):
            depth += {"<": 1, ">": -1}.get(n[j], 0)
            if depth == 0:
                end = j + 1
                break
    return n[m.start():end].replace("dgs::(anonymous namespace)::", "")[:40]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--steps", type=int, default=100)
    a = p.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    g = [x for x in rows if "k_gather<16" in x[2] and "StridedSrc" in x[2]]
    t0, t1 = g[a.warmup - 1][1], g[a.warmup + a.steps - 1][1]
    win = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in sorted(win):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t1 - t0
    tot = sum(e - s for s, e, _ in win)
    gaps.sort()
    print(f"window {span / 1e3:.1f} us ({span / a.steps / 1e3:.1f} us/step), GPU busy "
          f"{busy / span:.1%}, summed kernel time {tot / span:.2f}x the window, "
          f"{len(win)} kernels ({len(win) / a.steps:.1f}/step), {len(gaps)} idle gaps, "
          f"total {sum(gaps) / 1e3:.1f} us, largest {[round(x / 1e3, 1) for x in gaps[-5:]]}")
    # the feature gather's own launches in the window (what bench.py's roofline.avg_launch_ms
    # measures with HIP events over the timed region)
    gw = [e - s for s, e, n in rows if "k_gather<16" in n and "StridedSrc" in n
          and s >= t0 and e <= t1]
    if gw:
        print(f"feature gather in the window: {len(gw)} launches, avg {sum(gw) / len(gw) / 1e3:.2f} us")
    per = {}
    for s, e, n in win:
        k = short_name(n)
        per[k] = per.get(k, 0) + e - s
    for k, v in sorted(per.items(), key=lambda x: -x[1])[:12]:
        print(f"  {k:42s} {v / a.steps / 1e3:8.1f} us/step")


if __name__ == "__main__":
    main()
