#!/bin/bash
# Round 4: lazy reservoir modulo (no final conditional subtract): exhaustive/random modulo fuzz
# of the exact and lazy forms, uniform GPU parity tests, same-box A/B (uniform, pipelined and
# sequential) against the build without it.
set -uo pipefail
N=${1:-r04i}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
echo "== $(date +%T) modfuzz"
timeout -k 10 600 ./tools/modfuzz all > $O/modfuzz.txt 2>&1; rc=$?; tail -8 $O/modfuzz.txt; ok $rc
bash tools/r04_run.sh $N pytest; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 900 python tools/ab_bench.py --rounds 4 -- $(v blat) $(v lazy) \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
echo "== end $(date +%T)"
