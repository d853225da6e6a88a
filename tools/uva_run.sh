#!/bin/bash
# partial HBM caches with the other rows read zero-copy from pinned host
# memory (bench.py --cache-frac), sequential loop and 3 batches in flight.  Run on the GPU box:
#   bash tools/uva_run.sh r02
set -euo pipefail
R=${1:-r02}
O=gpurun_out/$R/uva
mkdir -p $O
for f in 0 0.05 0.2 0.5; do
  for d in 1 3; do
    timeout -k 10 300 python bench.py --cache-frac $f --depth $d --steps 300 --no-cpu-baseline \
      > $O/u_${f}_d$d.log 2>&1
  done
done
timeout -k 10 300 python bench.py --cache-frac 0.2 --bias --depth 3 --steps 300 --no-cpu-baseline \
  > $O/b_0.2_d3.log 2>&1
for f in $O/*.log; do grep -h '^{' "$f" | tail -n 1; done > $O/lines.jsonl
