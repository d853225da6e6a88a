"""Per-hop average durations of the sampling kernels from a rocprofv3 kernel-trace CSV (the
sequential loop: kernels of one call cycle through hops 0..L-1; the last 600 launches are used)."""
import csv, sys, collections
def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        for key in ("k_bias_boot", "k_bias_stream", "k_bias_rows_merge", "k_bias_hub_merge", "k_sample_bias", "k_dcount"):
            if key + "(" in n or key + "<" in n:
                seq[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return seq
for p in sys.argv[1:]:
    s = load(p)
    print(p.split("/")[2])
    for key, v in s.items():
        v = v[-600:]  # steady part
        hops = [v[h::3] for h in range(3)]
        print(f"  {key:20s} " + "  ".join(f"hop{h} {sum(x)/len(x):6.1f}" for h, x in enumerate(hops)))
