#!/bin/bash
# Round 4 head check: all GPU tests, smoke, papers-like bias hub statistics before (ab/cur) and
# after the stream kernel's adaptive threshold (head), N = 2 shared-device bench, N = 1 bench.
set -uo pipefail
N=${1:-r04j}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
bash tools/r04_run.sh $N pytest smoke; ok $?
for lib in cur head; do
  echo "== $(date +%T) papers bias stats $lib"
  if [ $lib = head ]; then env=""; else env="DGS_AMD_LIB=ab/$lib/libdgs_amd.so DGS_BENCH_PYDIR=$PWD/ab/$lib/py"; fi
  env $env DGS_BIAS_STATS=1 timeout -k 10 400 python tools/r04_bias_stats.py --scale 27 --ef 12 \
    > $O/stats_$lib.txt 2>&1; rc=$?; grep -v amdgpu.ids $O/stats_$lib.txt | tail -8; ok $rc
done
bash tools/r04_run.sh $N n2 bench; ok $?
echo "== end $(date +%T)"
