#!/bin/bash
# Round 4 head check 3: the lane-move unit check (if it fails, the in-tree library is replaced by
# ab/ilp4, the same head without the DPP lane moves), GPU tests, smoke, bench lines, N = 2
# self-check, hub-kernel workgroup stamps inside the pipeline (DGS_PROF_HUB), parity with the
# uniform hub kernel's dynamic pools, and a same-box A/B of the biased merge / lane moves.
set -uo pipefail
O=gpurun_out/r04_head3
mkdir -p $O
L=dist-gnn_amd/lib/libdgs_amd.so
timeout -k 10 60 ./tools/lane_ops_test > $O/lane_ops.txt 2>&1; rc=$?; tail -12 $O/lane_ops.txt
case $rc in
  0) ;;
  1) echo "lane ops FAILED: HEAD without the lane moves (ab/ilp4)"; cp ab/ilp4/libdgs_amd.so $L ;;
  *) exit $rc ;;
esac
bash tools/r04_run.sh r04_head3 pytest smoke bench n2 bias papersbias || exit $?
for v in "" "--bias"; do
  DGS_PROF_HUB=1 DGS_PROF_DETAIL=1 timeout -k 10 300 python bench.py --no-cpu-baseline $v \
    > $O/hubstamps$v.json 2> $O/hubstamps$v.err || exit $?
  grep "dgs prof" $O/hubstamps$v.err | tail -4
done
DGS_HUB_DYN=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_fullsize_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_hubdyn8.log 2>&1 || exit $?
tail -2 $O/pytest_hubdyn8.log
AB_ROUNDS=3 AB_VARIANTS="ab/ilp1/libdgs_amd.so ab/ilp4/libdgs_amd.so $L" AB_ARGS="--bias" \
  bash tools/r04_run.sh r04_head3_biasab ab
