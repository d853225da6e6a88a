#!/bin/bash
# Round 4: k_bias_stream grid size after the LDS staging (DGS_BIAS_STREAM_BLOCKS 768 / 1024 /
# 1536), same-box A/B papers-like and products-like biased.
set -uo pipefail
N=${1:-r04r}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/lds/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/lds/py,DGS_BIAS_STREAM_BLOCKS=$1"; }
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v 768) $(v 1024) $(v 1536) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v 768) $(v 1024) $(v 1536) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== end $(date +%T)"
