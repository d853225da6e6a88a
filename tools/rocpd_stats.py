"""Per-kernel statistics from a rocprofv3 rocpd database (the default output of ROCm 7's
`rocprofv3 --kernel-trace --stats` when no --output-format is given): the same summary lines as
profiles/r0*_kernel_stats_summary.txt, and the same columns as rocprofv3's kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/<call>/prof/run_results.db [summary.txt [stats.csv]]
"""
import csv
import re
import sqlite3
import sys


def short(name):
    s = re.sub(r"^(void )?dgs::\(anonymous namespace\)::", "", name)
    s = re.sub(r"\(dgs::.*$", "", s)
    s = s.replace("dgs::(anonymous namespace)::", "").replace("dgs::", "")
    return s[:70]


def main():
    db = sys.argv[1]
    con = sqlite3.connect(db)
    rows = con.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
        "from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    lines = [f"{short(n):70s} calls={c:5d} avg={a / 1e3:9.1f}us max={mx / 1e3:9.1f}us "
             f"tot={t / 1e6:8.2f}ms" for n, c, t, a, mn, mx in rows]
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    else:
        sys.stdout.write(text)
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage",
                        "MinNs", "MaxNs"])
            for n, c, t, a, mn, mx in rows:
                w.writerow([n, c, t, f"{a:.1f}", f"{100.0 * t / total:.4f}", mn, mx])


if __name__ == "__main__":
    main()
