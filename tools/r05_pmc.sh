#!/bin/bash
# Round 5: the gather's HBM traffic counters (FETCH_SIZE / WRITE_SIZE, separate passes) under a
# bench workload and under the known-byte calibration gather of the same row width, then a
# profiles-ready gather_pmc JSON.  bash tools/r05_pmc.sh NAME DIM [bench args...]
set -uo pipefail
N=$1; DIM=$2; shift 2
O=gpurun_out/$N
mkdir -p $O
export TMPDIR=/tmp DGS_PMC_DIM=$DIM
B="bench.py --no-cpu-baseline --secondary none --steps 10 --warmup 2 --seq-calls 3 --dim $DIM $*"
for c in FETCH_SIZE WRITE_SIZE; do
  t=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_bench_$t -- python3 $B \
    > $O/pmc_bench_$t.log 2>&1 || { tail -5 $O/pmc_bench_$t.log; exit 1; }
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_calib_$t -- python3 \
    tools/gather_calib.py > $O/pmc_calib_$t.log 2>&1 || { tail -5 $O/pmc_calib_$t.log; exit 1; }
done
python3 tools/pmc_traffic.py $O $O/gather_pmc_d$DIM.json > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
cat $O/gather_pmc_d$DIM.json
