import csv, re, sys
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
tot = 0
out = []
for r in rows:
    n = r['Name']
    m = re.search(r'(k_\w+)(<[^()]*>)?', n)
    short = (m.group(1) + (m.group(2) or '')) if m and 'dgs' in n else n[:50]
    out.append((float(r['TotalDurationNs']), short, int(r['Calls']), float(r['AverageNs']), float(r['MaxNs'])))
for t, nm, c, a, mx in sorted(out, reverse=True)[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{nm[:70]:70s} calls={c:5d} avg={a/1e3:9.1f}us max={mx/1e3:9.1f}us tot={t/1e6:8.2f}ms")
