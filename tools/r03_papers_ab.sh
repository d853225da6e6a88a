#!/bin/bash
# configs[3] shape (papers100M-like RMAT scale 27 x ef 12, d = 128, degree-weighted biased,
# [15,10,5]) same-box A/B of the given variants (tools/ab_bench.py), 2 rounds.
#   bash tools/r03_papers_ab.sh OUT variantA variantB ...
set -uo pipefail
O=gpurun_out/$1
shift
mkdir -p $O
echo "== $(date +%T) papers A/B"
AB_TIMEOUT=500 timeout -k 10 1100 python tools/ab_bench.py --rounds 2 -- "$@" -- --scale 27 --ef 12 \
  --dim 128 --bias --steps 200 --warmup 10 --seq-calls 20 > $O/ab_papers.txt 2>&1 \
  || { tail -20 $O/ab_papers.txt; exit 1; }
grep MEDIAN $O/ab_papers.txt
