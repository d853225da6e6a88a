#!/bin/bash
# Same-box uniform A/B of library builds: products-like (configs[1]) and papers100M-like.
#   bash tools/r03_uniform_ab.sh OUT libA libB ...
set -uo pipefail
O=gpurun_out/$1
shift
mkdir -p $O
echo "== $(date +%T) products"
timeout -k 10 600 python tools/ab_bench.py --rounds 3 -- "$@" > $O/ab_products.txt 2>&1 \
  || { tail -20 $O/ab_products.txt; exit 1; }
grep MEDIAN $O/ab_products.txt
echo "== $(date +%T) papers"
AB_TIMEOUT=400 timeout -k 10 900 python tools/ab_bench.py --rounds 2 -- "$@" -- --scale 27 --ef 12 \
  --dim 128 --steps 300 --seq-calls 20 > $O/ab_papers.txt 2>&1 || { tail -20 $O/ab_papers.txt; exit 1; }
grep MEDIAN $O/ab_papers.txt
echo "== $(date +%T) end"
