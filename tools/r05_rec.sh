#!/bin/bash
# round 5: biased hub-row records (k_bias_stream's row switch) -- parity + same-box A/B
O=gpurun_out/$1; mkdir -p $O
export DGS_AMD_LIB=$PWD/ab/rec/libdgs_amd.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "bias" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
unset DGS_AMD_LIB
timeout -k 10 500 python tools/ab_bench.py --rounds 3 -- ab/gu/libdgs_amd.so ab/rec/libdgs_amd.so \
  -- --scale 27 --ef 12 --dim 128 --bias --steps 300 --secondary none > $O/ab_papers.txt 2>&1 \
  || { tail -20 $O/ab_papers.txt; exit 1; }
grep MEDIAN $O/ab_papers.txt
timeout -k 10 400 python tools/ab_bench.py --rounds 3 -- ab/gu/libdgs_amd.so ab/rec/libdgs_amd.so \
  -- --bias --steps 300 --secondary none > $O/ab_products.txt 2>&1 \
  || { tail -20 $O/ab_products.txt; exit 1; }
grep MEDIAN $O/ab_products.txt
