#!/bin/bash
# Biased parity tests with each library build given, then a same-box A/B of all of them
# (products-like, degree-weighted, B = 1024, 300 steps) and per-hop kernel durations of the first
# and last build (sequential loop).   bash tools/r03_ab_variants.sh OUT libA.so libB.so ...
set -uo pipefail
O=gpurun_out/$1
shift
mkdir -p $O
R="$GRAFT_REPO_ROOT"
for lib in "$@"; do
  [ "$lib" = "${1}" ] && continue  # the first build is the baseline (tested at its commit)
  n=$(basename $lib .so)
  echo "== $(date +%T) parity $n"
  DGS_AMD_LIB="$R/$lib" timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "bias or papers" > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 1; }
  tail -1 $O/pytest_$n.log
done
echo "== $(date +%T) A/B"
timeout -k 10 1200 python tools/ab_bench.py --rounds 3 -- "$@" -- --bias --steps 300 > $O/ab.txt 2>&1 \
  || { tail -20 $O/ab.txt; exit 1; }
grep MEDIAN $O/ab.txt
