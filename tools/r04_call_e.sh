#!/bin/bash
# Round 4 call: GPU tests at the head, the synchronous call's host breakdown, same-box A/B of
# round 3 / the first round-4 commit / the head (uniform), and of the first round-4 commit / the
# head (biased: the stream kernel's adaptive threshold).
set -uo pipefail
N=${1:-r04e}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
bash tools/r04_run.sh $N pytest synchost; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v r03) $(v cur) $(v new) \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
echo "== $(date +%T) ab bias"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v cur) $(v new) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== end $(date +%T)"
