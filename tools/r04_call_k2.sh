#!/bin/bash
# Round 4 call k2: lane-move unit check, biased parity with the lane moves and sorted first
# groups (HEAD), uniform hub A/B (ab/pre = bd82fbd, before the stamps / pools; HEAD with 0, 4, 8
# sixteenths in pools; 1024 workgroups), biased A/B (ab/ilp4 = merge ILP only, HEAD).
set -uo pipefail
O=gpurun_out/r04_k2
mkdir -p $O
L=dist-gnn_amd/lib/libdgs_amd.so
timeout -k 10 60 ./tools/lane_ops_test > $O/lane_ops.txt 2>&1; lrc=$?; tail -14 $O/lane_ops.txt
case $lrc in 0|1) ;; *) exit $lrc ;; esac
if [ $lrc -eq 0 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_papers_gpu.py \
    tests/test_prefetch_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_bias.log 2>&1
  prc=$?; tail -3 $O/pytest_bias.log; case $prc in 0|1) ;; *) exit $prc ;; esac
fi
AB_ROUNDS=3 AB_VARIANTS="ab/pre/libdgs_amd.so $L $L,DGS_HUB_DYN=4 $L,DGS_HUB_DYN=8 $L,DGS_HUB_BLOCKS=1024" \
  bash tools/r04_run.sh r04_k2_hubab ab || exit $?
if [ $lrc -eq 0 ] && [ ${prc:-1} -eq 0 ]; then
  AB_ROUNDS=3 AB_VARIANTS="ab/ilp4/libdgs_amd.so $L" AB_ARGS="--bias" bash tools/r04_run.sh r04_k2_biasab ab
fi
# biased stream kernel with dynamic pools (ab/bdyn = HEAD + pools in k_bias_stream, DGS_BIAS_DYN)
DGS_AMD_LIB=$PWD/ab/bdyn/libdgs_amd.so DGS_BIAS_DYN=8 timeout -k 10 600 python -u -m pytest \
  tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k bias \
  > $O/pytest_bdyn8.log 2>&1; brc=$?; tail -2 $O/pytest_bdyn8.log; case $brc in 0|1) ;; *) exit $brc ;; esac
if [ $brc -eq 0 ]; then
  B=ab/bdyn/libdgs_amd.so
  AB_ROUNDS=3 AB_VARIANTS="$B $B,DGS_BIAS_DYN=4 $B,DGS_BIAS_DYN=8" AB_ARGS="--bias" \
    bash tools/r04_run.sh r04_k2_bdynab ab
fi
