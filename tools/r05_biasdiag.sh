#!/bin/bash
# Round 5: per-kernel durations of the sequential biased call (kernel trace) and the biased hub
# statistics per hop (DGS_BIAS_STATS=1), for each library given.  bash tools/r05_biasdiag.sh NAME lib...
set -uo pipefail
N=$1; shift
O=gpurun_out/$N
mkdir -p $O
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  DGS_AMD_LIB=$(realpath $lib) DGS_BIAS_STATS=1 timeout -k 10 200 python3 bench.py --bias --steps 3 \
    --warmup 1 --depth 1 --seq-calls 3 --no-cpu-baseline --secondary none ${DIAG_ARGS:-} \
    > $O/stats_$i.json 2> $O/stats_$i.err || { tail -5 $O/stats_$i.err; exit 1; }
  grep "bias stats" $O/stats_$i.err | tail -6
  DGS_AMD_LIB=$(realpath $lib) timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
    -d $O/calls_$i -- python3 bench.py --bias --depth 1 --steps 100 --warmup 10 --seq-calls 3 \
    --no-cpu-baseline --secondary none ${DIAG_ARGS:-} > $O/calls_$i.log 2>&1 || { tail -5 $O/calls_$i.log; exit 1; }
  python3 tools/call_breakdown.py "$(ls -t $(find $O/calls_$i -name '*kernel_trace.csv') | head -n 1)" \
    > $O/call_breakdown_$i.txt; echo "== $lib"; tail -25 $O/call_breakdown_$i.txt
done
