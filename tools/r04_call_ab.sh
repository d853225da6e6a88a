#!/bin/bash
# Round 4: uniform hub reservoir with its row bookkeeping wave-uniform (chunk arithmetic on the
# scalar unit) and d = idx + 1 formed once per draw (ab/hubu, in-tree) against HEAD (ab/balign):
# GPU parity tests, same-box A/B of the default line (configs[1]) and B = 8192.
set -uo pipefail
N=${1:-r04ab}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py${2:+,$2}"; }
bash tools/r04_run.sh $N pytest:tests/test_gpu_parity.py pytest:tests/test_fullsize_gpu.py; ok $?
echo "== $(date +%T) ab uniform"
timeout -k 10 900 python tools/ab_bench.py --rounds 5 -- $(v hubu) $(v balign) -- \
  > $O/ab_uniform.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform.txt; ok $rc
echo "== $(date +%T) ab uniform B=8192"
timeout -k 10 900 python tools/ab_bench.py --rounds 3 -- $(v hubu) $(v balign) -- --batch 8192 \
  > $O/ab_uniform_b8192.txt 2>&1; rc=$?; grep MEDIAN $O/ab_uniform_b8192.txt; ok $rc
echo "== end $(date +%T)"
