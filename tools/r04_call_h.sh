#!/bin/bash
# Round 4: biased latency layout (non-hub rows beside the stream kernel, hub merge after) and the
# stream kernel's adaptive threshold: biased GPU tests; same-box A/B products-like; papers-like
# (configs[3] graph) hub statistics before / after the adaptive threshold and an A/B.
set -uo pipefail
N=${1:-r04h}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_prefetch_gpu.py; ok $?
echo "== $(date +%T) ab bias products"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v new2) $(v blat) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
for lib in cur blat; do
  echo "== $(date +%T) papers bias stats $lib"
  DGS_BIAS_STATS=1 DGS_AMD_LIB=ab/$lib/libdgs_amd.so DGS_BENCH_PYDIR=$PWD/ab/$lib/py \
    timeout -k 10 400 python tools/r04_bias_stats.py --scale 27 --ef 12 > $O/stats_$lib.txt 2>&1
  rc=$?; grep -v amdgpu.ids $O/stats_$lib.txt | tail -8; ok $rc
done
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1500 python tools/ab_bench.py --rounds 1 -- $(v new2) $(v blat) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== end $(date +%T)"
