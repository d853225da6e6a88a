"""Per-position kernel durations and gaps of the synchronous sample calls in a rocprofv3 rocpd
database (`rocprofv3 --kernel-trace -d D -o O -- python3 tools/sync_call_phases.py`): every call
is the chain of launches that starts at a k_prep of one 256-row tile grid (B = 1024 seeds: grid
1024 threads); calls with the modal launch count are kept and each position's median duration
and median gap to the previous launch are printed, with the call's median span.

    python tools/call_positions.py gpurun_out/<dir>/<name>_results.db [prep_grid]
"""
import collections
import re
import sqlite3
import statistics as st
import sys


def short(name):
    m = re.search(r"::(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:40]


def main():
    db = sys.argv[1]
    prep_grid = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, duration, grid_x, start, end from kernels "
                          "where name like '%dgs::%' order by start"))
    ks = [(short(n), d / 1e3, g, s, e) for n, d, g, s, e in rows]
    calls, cur = [], None
    for x in ks:
        if x[0] == "k_prep" and x[2] == prep_grid:
            if cur:
                calls.append(cur)
            cur = []
        if cur is not None:
            cur.append(x)
    if cur:
        calls.append(cur)
    if not calls:
        sys.exit("no calls found")
    n = collections.Counter(len(q) for q in calls).most_common(1)[0][0]
    calls = [q for q in calls if len(q) == n]
    print(f"{len(calls)} calls of {n} launches ({db})")
    for i in range(n):
        ds = [q[i][1] for q in calls]
        gaps = [(q[i][3] - q[i - 1][4]) / 1e3 for q in calls] if i else [0.0]
        print(f"  {calls[0][i][0]:42s} grid {calls[0][i][2]:8d} {st.median(ds):7.2f} us"
              f"   gap before {st.median(gaps):6.2f} us")
    print(f"  span {st.median([(q[-1][4] - q[0][3]) / 1e3 for q in calls]):.1f} us, kernels "
          f"{st.median([sum(x[1] for x in q) for q in calls]):.1f} us (medians)")


if __name__ == "__main__":
    main()
