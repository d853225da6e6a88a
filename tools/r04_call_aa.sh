#!/bin/bash
# Round 4: the biased rows + merge launch with 1024-thread workgroups (32 half-waves per hub row's
# merge; ab/mhw32, in-tree) or 512 (ab/mhw16) against HEAD's 256 (ab/balign): biased GPU tests,
# same-box A/B products-like and papers-like biased.
set -uo pipefail
N=${1:-r04aa}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py${2:+,$2}"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_papers_gpu.py pytest:tests/test_prefetch_gpu.py; ok $?
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v mhw32) $(v mhw16) $(v balign) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v mhw32) $(v mhw16) $(v balign) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
