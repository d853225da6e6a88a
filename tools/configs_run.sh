#!/bin/bash
# BASELINE configs[0] / configs[4] shaped runs on one MI355X (plus a biased kernel profile):
#   gpurun -- 'bash tools/configs_run.sh r01'
set -euo pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
# configs[0] shape: arxiv-like RMAT (scale 17, ef 9), fan-out [10,10], d=128
timeout -k 10 300 python bench.py --scale 17 --ef 9 --dim 128 --fan-out 10,10 > $O/bench_arxiv.log 2>&1
# configs[4] shape: RMAT-1B (scale 26, ef 16: 67 M nodes, 1.07 B edges), d=256, one GPU
timeout -k 10 900 python bench.py --scale 26 --ef 16 --dim 256 > $O/bench_rmat1b.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_bias -- python3 bench.py --bias --no-cpu-baseline --depth 1 > $O/stats_bias.log 2>&1
