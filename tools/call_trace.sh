#!/bin/bash
# Kernel trace of the sequential loop (one batch at a time) and the per-call breakdown
# (tools/call_breakdown.py), uniform and biased.  Run on the GPU box:
#   bash tools/call_trace.sh r02
set -euo pipefail
R=${1:-r02}
O=gpurun_out/$R/calls
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in uniform bias; do
  extra=""
  [ $v = bias ] && extra="--bias"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$v -- \
    python3 bench.py --depth 1 --steps 100 --warmup 10 --no-cpu-baseline $extra > $O/$v.log 2>&1
  python3 tools/call_breakdown.py "$(ls -t $(find $O/$v -name '*kernel_trace.csv') | head -n 1)" > $O/$v.txt
done
