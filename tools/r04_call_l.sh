#!/bin/bash
# Round 4: uniform hub reservoir with chunk pairs (four Philox blocks in flight): parity tests,
# same-box A/B against the head without it (B = 1024 and 8192; pipelined and sequential).
set -uo pipefail
N=${1:-r04l}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_fullsize_gpu.py; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 600 python tools/ab_bench.py --rounds 4 -- $(v head) $(v pairs) \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
echo "== $(date +%T) ab uniform B=8192"
timeout -k 10 600 python tools/ab_bench.py --rounds 3 -- $(v head) $(v pairs) -- --batch 8192 \
  > $O/ab_uniform_8192.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform_8192.txt; ok $rc
echo "== end $(date +%T)"
