#!/bin/bash
# Round 4: stream chunks aligned to each lane's Philox blocks (no draw window, no carried block)
# and the round keys computed once per row (ab/salign, in-tree) against HEAD (ab/svalid): all GPU
# tests, same-box A/B products-like and papers-like biased.
set -uo pipefail
N=${1:-r04y}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py${2:+,$2}"; }
bash tools/r04_run.sh $N pytest; ok $?
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v salign) $(v svalid) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v salign) $(v svalid) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
