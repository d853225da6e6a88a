#!/bin/bash
# BASELINE configs[3] shape on one MI355X: papers100M-like RMAT (scale 27 x ef 12: 134 M nodes,
# 1.61 B edges), d = 128, fan-out [15,10,5], uniform and degree-weighted biased:
#   gpurun -- 'bash tools/papers_run.sh r01'
set -euo pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 900 python bench.py --scale 27 --ef 12 --dim 128 > $O/bench_papers_uniform.log 2>&1
timeout -k 10 900 python bench.py --scale 27 --ef 12 --dim 128 --bias > $O/bench_papers_bias.log 2>&1
