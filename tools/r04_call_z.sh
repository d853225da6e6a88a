#!/bin/bash
# Round 4: the boot on whole Philox blocks (runs cut at block boundaries, round keys once,
# 32-bit indices, one-address loads; ab/balign) and the same with the reciprocal key bound
# (ab/bklow, in-tree) against HEAD (ab/salign): biased GPU tests (incl. the bound soundness
# test, run on the in-tree bklow build), same-box A/B products-like and papers-like biased.
set -uo pipefail
N=${1:-r04z}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py${2:+,$2}"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_papers_gpu.py pytest:tests/test_prefetch_gpu.py; ok $?
echo "== $(date +%T) parity of ab/balign"
DGS_AMD_LIB=ab/balign/libdgs_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "bias" \
  --timeout 120 --timeout-method thread > $O/pytest_balign.log 2>&1; rc=$?; tail -2 $O/pytest_balign.log; ok $rc
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v bklow) $(v balign) $(v salign) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v bklow) $(v balign) $(v salign) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
