#!/bin/bash
# Round-3 bench lines of every BASELINE config shape on one MI355X (each step its own limit):
#   part a: configs[0] arxiv-like, configs[1] products-like uniform / biased at B = 1024 and 8192
#   part b: configs[3] papers100M-like uniform / biased, configs[4] RMAT-1B
set -uo pipefail
O=gpurun_out/$1
PART=$2
mkdir -p $O
run() {  # name, limit, args...
  local n=$1 t=$2; shift 2
  echo "== $(date +%T) $n"
  timeout -k 10 $t python bench.py "$@" > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
}
if [ "$PART" = a ]; then
  run arxiv 300 --scale 17 --ef 9 --dim 128 --fan-out 10,10 --no-cpu-baseline
  run products_bias 300 --bias --no-cpu-baseline
  run products_b8192 300 --batch 8192 --no-cpu-baseline
  run products_b8192_bias 300 --batch 8192 --bias --no-cpu-baseline
else
  run papers_uniform 600 --scale 27 --ef 12 --dim 128 --no-cpu-baseline
  run papers_bias 600 --scale 27 --ef 12 --dim 128 --bias --no-cpu-baseline
  run rmat1b 600 --scale 26 --ef 16 --dim 256 --no-cpu-baseline
fi
echo "== $(date +%T) end"
