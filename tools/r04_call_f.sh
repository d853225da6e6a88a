#!/bin/bash
# Round 4: loader seeds read one batch ahead (batch streams wait on the seeds' event, not on the
# caller's tail): loader tests, then same-box A/B round 3 / before / after (uniform pipelined).
set -uo pipefail
N=${1:-r04f}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
bash tools/r04_run.sh $N pytest:tests/test_loader_order_gpu.py pytest:tests/test_prefetch_gpu.py; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v r03) $(v new) $(v new2) \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
bash tools/r04_run.sh $N pmcpipe calltrace; ok $?
echo "== end $(date +%T)"
