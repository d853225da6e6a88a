"""Summaries of rocprofv3 `--stats` kernel tables.

    python tools/prof_summary.py <kernel_stats.csv> [N]          top-N kernels by total time
    python tools/prof_summary.py --compare <a.csv> <b.csv> ...   DGS kernels side by side
"""
import csv
import re
import sys


def load(path):
    out = {}
    for r in csv.DictReader(open(path)):
        n = r['Name'].replace('dgs::(anonymous namespace)::', '')
        m = re.search(r'(k_\w+)(<.*?>)?(?=\(|$)', n)
        short = (m.group(1) + (m.group(2) or '')) if m and 'dgs' in r['Name'] else n[:50]
        t, c, mx = float(r['TotalDurationNs']), int(r['Calls']), float(r['MaxNs'])
        if short in out:
            t0, c0, mx0 = out[short]
            out[short] = (t0 + t, c0 + c, max(mx0, mx))
        else:
            out[short] = (t, c, mx)
    return out


def main():
    if sys.argv[1] == '--compare':
        tabs = [load(p) for p in sys.argv[2:]]
        names = sorted({n for t in tabs for n in t if n.startswith('k_')},
                       key=lambda n: -tabs[0].get(n, (0, 1, 0))[0])
        print(f"{'kernel (avg us)':44s}" + ''.join(f"{i:>10d}" for i in range(len(tabs))))
        for n in names:
            cells = []
            for t in tabs:
                v = t.get(n)
                cells.append(f"{v[0] / v[1] / 1e3:10.2f}" if v else f"{'-':>10s}")
            print(f"{n[:44]:44s}" + ''.join(cells))
        return
    out = sorted(((t, n, c, t / c, mx) for n, (t, c, mx) in load(sys.argv[1]).items()),
                 reverse=True)
    for t, nm, c, a, mx in out[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
        print(f"{nm[:70]:70s} calls={c:5d} avg={a/1e3:9.1f}us max={mx/1e3:9.1f}us tot={t/1e6:8.2f}ms")


if __name__ == '__main__':
    main()
