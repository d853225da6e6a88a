#!/bin/bash
# Round 4: papers-like biased hub statistics (candidate spread) and a kernel trace of the
# synchronous call with the rows part and the hub merge as separate launches.
set -uo pipefail
N=${1:-r04p}
O=gpurun_out/$N
mkdir -p $O
DGS_BIAS_STATS=1 timeout -k 10 400 python tools/r04_bias_stats.py --scale 27 --ef 12 \
  > $O/stats.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/stats.txt | tail -8; [ $rc -le 1 ] || exit $rc
DGS_BIAS_SPLIT_MERGE=1 CALL_ARGS="--bias --scale 27 --ef 12 --dim 128" bash tools/r04_run.sh $N calltrace || exit $?
rm -rf $O/calls
