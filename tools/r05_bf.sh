#!/bin/bash
# round 5: bf16 upper-bound probabilities for the biased stream filter -- GPU tests, then A/B
O=gpurun_out/$1; mkdir -p $O
bash tools/r05_run.sh $1 pytest | tail -2
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" <(tail -1 $O/pytest.log) || exit 1
timeout -k 10 500 python tools/ab_bench.py --rounds 3 -- ab/cur/libdgs_amd.so ab/bf/libdgs_amd.so \
  -- --bias --steps 300 --secondary none > $O/ab_products_bias.txt 2>&1 || { tail -5 $O/ab_products_bias.txt; exit 1; }
grep MEDIAN $O/ab_products_bias.txt
AB_TIMEOUT=400 timeout -k 10 600 python tools/ab_bench.py --rounds 3 -- ab/cur/libdgs_amd.so ab/bf/libdgs_amd.so \
  -- --scale 27 --ef 12 --dim 128 --bias --steps 300 --secondary none > $O/ab_papers_bias.txt 2>&1 || { tail -5 $O/ab_papers_bias.txt; exit 1; }
grep MEDIAN $O/ab_papers_bias.txt
