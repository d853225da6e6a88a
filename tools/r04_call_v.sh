#!/bin/bash
# Round 4: SQ counters per kernel of the biased sequential loop (rocprofv3 serialises kernels
# under --pmc, so the counters are per kernel alone), products-like and papers-like.
set -uo pipefail
N=${1:-r04v}
O=gpurun_out/$N
mkdir -p $O
export TMPDIR=/tmp
ok() { case $1 in 0|1) return 0 ;; *) echo "stop: rc=$1"; exit $1 ;; esac; }
for cfg in products papers; do
  args="--bias"; [ $cfg = papers ] && args="--bias --scale 27 --ef 12 --dim 128"
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU \
    --output-format csv -d $O/pmc_$cfg -- python3 bench.py --depth 1 --steps 30 \
    --warmup 3 --seq-calls 1 --no-cpu-baseline $args > $O/pmc_$cfg.log 2>&1; rc=$?
  ok $rc
  python3 tools/pmc_kernels.py "$(find $O/pmc_$cfg -name '*counter_collection.csv' | head -n 1)" \
    > $O/pmc_${cfg}_summary.txt; head -14 $O/pmc_${cfg}_summary.txt | cut -c1-300
  rm -rf $O/pmc_$cfg
done
