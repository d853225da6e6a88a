#!/bin/bash
# Round 4: the boot's key lower bound from one reciprocal, (u - 1) / (u p ln 2), instead of the
# hardware log2 + reciprocal (ab/klow, the in-tree build) against HEAD (ab/lds): biased GPU
# tests (incl. the bound soundness test), candidate statistics, same-box A/B.
set -uo pipefail
N=${1:-r04u}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py${2:+,$2}"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_papers_gpu.py; ok $?
for lib in klow lds; do
  echo "== $(date +%T) products bias stats $lib"
  DGS_BIAS_STATS=1 DGS_AMD_LIB=ab/$lib/libdgs_amd.so DGS_BENCH_PYDIR=$PWD/ab/$lib/py \
    timeout -k 10 300 python tools/r04_bias_stats.py > $O/stats_products_$lib.txt 2>&1
  rc=$?; grep "bias stats" $O/stats_products_$lib.txt | tail -4; ok $rc
done
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 5 -- $(v klow) $(v lds) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v klow) $(v lds) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
