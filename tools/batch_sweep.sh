#!/bin/bash
# Pipelined throughput over the batch size (products-like graph, uniform and biased): one bench
# line per (sampler, B).  Run on the GPU box:  bash tools/batch_sweep.sh r02
set -euo pipefail
R=${1:-r02}
O=gpurun_out/$R/sweep
mkdir -p $O
for b in 256 512 1024 2048 4096 8192 16384; do
  timeout -k 10 300 python bench.py --batch $b --steps 300 --no-cpu-baseline > $O/u_$b.log 2>&1
  timeout -k 10 300 python bench.py --batch $b --steps 300 --no-cpu-baseline --bias > $O/b_$b.log 2>&1
done
python - "$O" <<'PY' > $O/summary.jsonl
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log")), key=lambda p: (p.split("/")[-1][0], int(p.split("_")[-1][:-4]))):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(json.dumps({"sampler": "biased" if "/b_" in f else "uniform", "batch": d["config"]["batch_per_gpu"],
                      "sampled_edges_per_s": d["value"], "ms_per_step": d["ms_per_step"],
                      "edges_per_step": d["sampled_edges_per_step"],
                      "gather_frac_pipeline": d["roofline"]["frac"],
                      "gather_frac_isolated": d["roofline_isolated"]["frac"],
                      "sample_span_ms": d["sample_span_ms_per_call"]}))
PY
