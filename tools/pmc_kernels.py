"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (DGS kernels only), plus
VALU instructions per wave and the share of wave cycles with a VALU instruction in flight
(SQ_ACTIVE_INST_VALU and SQ_WAVE_CYCLES both count quad-cycles)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for r in rows:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("dgs::", "")
    n = n.replace("void ", "").split("(")[0]
    if not n.startswith("k_"):
        continue
    agg[n][r["Counter_Name"]] += float(r["Counter_Value"])
    launches[n].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
for n, d in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    c = max(len(launches[n]), 1)
    waves = d.get("SQ_WAVES", 0) / c
    line = f"{n:34s} launches={c:5d} waves/launch={waves:9.0f}"
    if waves:
        line += f" VALU/wave={d.get('SQ_INSTS_VALU', 0) / c / waves:8.0f}"
        line += f" SALU/wave={d.get('SQ_INSTS_SALU', 0) / c / waves:7.0f}"
        line += f" LDS/wave={d.get('SQ_INSTS_LDS', 0) / c / waves:6.0f}"
    if d.get("SQ_WAVE_CYCLES"):
        wc = d["SQ_WAVE_CYCLES"]
        line += f" VALU-active/wave-cycles={d.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}"
        if waves:
            line += f" wave-cycles/wave={wc / c / waves:8.0f}"
        for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
            if k in d:
                line += f" {k[3:].lower()}/wave-cycles={d[k] / wc:.3f}"
    known = {"SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
             "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"}
    for k in sorted(d):  # any other counter: its per-launch average
        if k not in known:
            line += f" {k}/launch={d[k] / c:.4g}"
    print(line)
