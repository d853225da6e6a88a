#!/bin/bash
# round 5: two-chunk-deep probability prefetch in k_bias_stream -- biased parity, then A/B
O=gpurun_out/$1; mkdir -p $O
DGS_AMD_LIB=$PWD/ab/pf2/libdgs_amd.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_papers_gpu.py \
  tests/test_prefetch_gpu.py -k "bias or papers or prefetch" > $O/pytest_pf2.log 2>&1 \
  || { tail -30 $O/pytest_pf2.log; exit 1; }
tail -1 $O/pytest_pf2.log
timeout -k 10 500 python tools/ab_bench.py --rounds 3 -- ab/cur/libdgs_amd.so ab/pf2/libdgs_amd.so \
  -- --bias --steps 300 --secondary none > $O/ab_products_bias.txt 2>&1 || { tail -5 $O/ab_products_bias.txt; exit 1; }
grep MEDIAN $O/ab_products_bias.txt
AB_TIMEOUT=400 timeout -k 10 600 python tools/ab_bench.py --rounds 3 -- ab/cur/libdgs_amd.so ab/pf2/libdgs_amd.so \
  -- --scale 27 --ef 12 --dim 128 --bias --steps 300 --secondary none > $O/ab_papers_bias.txt 2>&1 || { tail -5 $O/ab_papers_bias.txt; exit 1; }
grep MEDIAN $O/ab_papers_bias.txt
