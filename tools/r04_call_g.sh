#!/bin/bash
# Round 4: latency layout of the synchronous call (non-hub rows beside the hub reservoir):
# GPU tests, call trace, same-box A/B (pipelined + sequential) against the previous head, and
# the latency layout forced into the pipeline.
set -uo pipefail
N=${1:-r04g}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
bash tools/r04_run.sh $N pytest calltrace synchost; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v new2) $(v lat) $(v lat),DGS_LATENCY_LAYOUT=1 \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
echo "== end $(date +%T)"
