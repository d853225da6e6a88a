#!/bin/bash
# The N = 2 shared-GPU rehearsal under three launch variants (default pipelined loader,
# launches on the caller's thread, the sequential loop).  A variant that fails with an ordinary
# error (exit 1) does not stop the next one; a fault, abort or time limit ends the script.
set -uo pipefail
O=gpurun_out/${1:-r03n2}
mkdir -p $O
run() {
  local name=$1; shift
  echo "== $(date +%T) $name"
  env "$@" DGS_BENCH_SHARE_DEVICE=1 timeout -k 10 240 python bench.py --gpus 2 --steps 100 \
    --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-} > $O/$name.log 2>&1
  local rc=$?
  grep -h "internal error\|^{" $O/$name.log | cut -c1-400
  echo "rc=$rc"
  case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
run default X=1
run sync DGS_PREFETCH_SYNC=1
BENCH_EXTRA="--depth 1" run depth1 X=1
echo "== end"
