#!/bin/bash
# SQ counters of the biased kernels for two library builds (products-like, degree-weighted,
# sequential loop):  bash tools/r03_pmc_ab.sh OUT libA.so libB.so
set -uo pipefail
O=gpurun_out/$1
shift
mkdir -p $O
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp && cd "$R"
B="bench.py --bias --depth 1 --no-cpu-baseline --steps 50 --warmup 5 --seq-calls 5"
for lib in "$@"; do
  n=$(basename $lib .so)
  echo "== $(date +%T) $n"
  DGS_AMD_LIB="$R/$lib" timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_$n -- python3 $B > $O/pmc_$n.log 2>&1 || { tail -5 $O/pmc_$n.log; exit 1; }
  python3 tools/pmc_kernels.py "$(find $O/pmc_$n -name '*counter_collection.csv' | head -n 1)" > $O/pmc_$n.txt
  grep -E "k_bias" $O/pmc_$n.txt
done
