#!/bin/bash
# round 5: uniform row-kernel group size (lanes per row) -- parity then same-box A/B
O=gpurun_out/$1; mkdir -p $O
for g in ${GROUPS_UNDER_TEST:-g8 g4}; do
  DGS_AMD_LIB=$PWD/ab/$g/libdgs_amd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_fullsize_gpu.py \
    > $O/pytest_$g.log 2>&1 || { tail -30 $O/pytest_$g.log; exit 1; }
  tail -1 $O/pytest_$g.log
done
timeout -k 10 700 python tools/ab_bench.py --rounds 5 -- ab/solo/libdgs_amd.so \
  $(for g in ${GROUPS_UNDER_TEST:-g8 g4}; do echo ab/$g/libdgs_amd.so; done) -- --secondary none > $O/ab.txt 2>&1 \
  || { tail -20 $O/ab.txt; exit 1; }
grep MEDIAN $O/ab.txt
