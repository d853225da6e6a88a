#!/bin/bash
# The gather's HBM traffic counters (FETCH_SIZE / WRITE_SIZE, separate passes) under the bench and
# under the known-byte calibration gather, then profiles-ready gather_pmc.json.
set -uo pipefail
O=gpurun_out/${1:-r03pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --no-cpu-baseline --steps 10 --warmup 2"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench_fetch -- python3 $B > $O/pmc_bench_fetch.log 2>&1 || { tail -5 $O/pmc_bench_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_bench_write -- python3 $B > $O/pmc_bench_write.log 2>&1 || { tail -5 $O/pmc_bench_write.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_calib_fetch -- python3 tools/gather_calib.py > $O/pmc_calib_fetch.log 2>&1 || { tail -5 $O/pmc_calib_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_calib_write -- python3 tools/gather_calib.py > $O/pmc_calib_write.log 2>&1 || { tail -5 $O/pmc_calib_write.log; exit 1; }
python tools/pmc_traffic.py $O $O/gather_pmc.json > $O/pmc_traffic.log 2>&1 || { tail -5 $O/pmc_traffic.log; exit 1; }
cat $O/gather_pmc.json
