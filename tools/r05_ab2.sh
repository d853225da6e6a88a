#!/bin/bash
# two same-box A/Bs in one call: products-like uniform (1000 steps) and papers-like biased
# (300 steps).  bash tools/r05_ab2.sh NAME "variants"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 700 python tools/ab_bench.py --rounds ${AB_ROUNDS:-3} -- $2 -- --secondary none \
  > $O/ab_uniform.txt 2>&1 || { tail -20 $O/ab_uniform.txt; exit 1; }
grep MEDIAN $O/ab_uniform.txt
AB_TIMEOUT=400 timeout -k 10 900 python tools/ab_bench.py --rounds ${AB_ROUNDS:-3} -- $2 -- \
  --scale 27 --ef 12 --dim 128 --bias --steps 300 --secondary none > $O/ab_papers.txt 2>&1 \
  || { tail -20 $O/ab_papers.txt; exit 1; }
grep MEDIAN $O/ab_papers.txt
