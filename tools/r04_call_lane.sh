#!/bin/bash
# Round 4: DPP / permlane16_swap lane moves in the half-wave top-k networks.  The lane-op unit
# check, the biased GPU parity tests under ab/lane, then a same-box A/B of the biased lines:
# ab/ilp1 (round-3 merge), HEAD (merge ILP 4), ab/lane (merge ILP 4 + DPP lane moves).
set -uo pipefail
O=gpurun_out/r04_lane
mkdir -p $O
timeout -k 10 60 ./tools/lane_ops_test > $O/lane_ops.txt 2>&1; rc=$?; cat $O/lane_ops.txt | tail -12
[ $rc -eq 0 ] || exit $rc
DGS_AMD_LIB=$PWD/ab/lane/libdgs_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py \
  tests/test_papers_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_lane.log 2>&1 || { tail -30 $O/pytest_lane.log; exit 1; }
tail -2 $O/pytest_lane.log
L=dist-gnn_amd/lib/libdgs_amd.so
AB_ROUNDS=${AB_ROUNDS:-3} AB_VARIANTS="ab/ilp1/libdgs_amd.so $L ab/lane/libdgs_amd.so" AB_ARGS="--bias" \
  bash tools/r04_run.sh r04_lane_ab ab || exit $?
AB_ROUNDS=1 AB_VARIANTS="ab/ilp1/libdgs_amd.so $L ab/lane/libdgs_amd.so" \
  AB_ARGS="--bias --scale 27 --ef 12 --dim 128 --steps 300" AB_TIMEOUT=600 bash tools/r04_run.sh r04_lane_ab_papers ab
