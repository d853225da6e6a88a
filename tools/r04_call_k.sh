#!/bin/bash
# Round 4: the stream kernel's adaptive threshold, same-box A/B before (ab/cur) / after (head):
# papers100M-like and products-like biased; then the driver's short run (20 timed steps after 5
# warm-up) three times at the head.
set -uo pipefail
N=${1:-r04k}
O=gpurun_out/$N
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
v() { echo "ab/$1/libdgs_amd.so,DGS_BENCH_PYDIR=$PWD/ab/$1/py"; }
echo "== $(date +%T) ab bias papers"
AB_TIMEOUT=600 timeout -k 10 1000 python tools/ab_bench.py --rounds 3 -- $(v cur) $(v head) -- \
  --bias --scale 27 --ef 12 --dim 128 --steps 300 > $O/ab_bias_papers.txt 2>&1; rc=$?
grep MEDIAN $O/ab_bias_papers.txt; ok $rc
echo "== $(date +%T) ab bias products"
timeout -k 10 600 python tools/ab_bench.py --rounds 3 -- $(v cur) $(v head) -- --bias \
  > $O/ab_bias.txt 2>&1; rc=$?; grep MEDIAN $O/ab_bias.txt; ok $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/short_$i.json \
    2> $O/short_$i.err; rc=$?; ok $rc
  python -c "import json; d=json.loads(open('$O/short_$i.json').read().strip().splitlines()[-1]); print('short', $i, round(d['value']/1e9,3), 'G', round(d['ms_per_step'],4), 'ms/step', d['host_step_gap_ms'])"
done
echo "== end $(date +%T)"
