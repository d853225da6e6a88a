#!/bin/bash
# Round 4, first GPU call: GPU tests (incl. the loader-order test), the N = 2 old/new probe,
# one N = 1 bench line at the round-3 head.
set -uo pipefail
O=gpurun_out/${1:-r04a}
mkdir -p $O
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
echo "== $(date +%T) pytest"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; ok $rc
echo "== $(date +%T) probe"
RUNS=${RUNS:-3} bash tools/r04_n2_probe.sh ${1:-r04a}/n2; ok $?
echo "== $(date +%T) bench"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
rc=$?; cat $O/bench.json | cut -c1-600; ok $rc
echo "== end $(date +%T)"
