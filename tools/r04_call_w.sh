#!/bin/bash
# Round 4: the stream kernel with raw compare masks, bit-field selects and one-address
# probability loads (ab/smask) against HEAD (ab/lds): biased GPU tests (incl. the bound
# soundness test), same-box A/B products-like and papers-like biased.
set -uo pipefail
N=${1:-r04w}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
A=${A:-smask}; B=${B:-lds}
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_papers_gpu.py; ok $?
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v $A) $(v $B) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v $A) $(v $B) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
