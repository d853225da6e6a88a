#!/bin/bash
# Biased stream kernel diagnostics (products-like, degree-weighted, sequential loop): SQ counters,
# HBM fetch bytes (FETCH_SIZE), and the hub edge rate from tools/hub_rate.py over a kernel trace.
set -uo pipefail
O=gpurun_out/${1:-r03bp}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="bench.py --bias --depth 1 --no-cpu-baseline --steps 50 --warmup 5 --seq-calls 5"
echo "== $(date +%T) sq"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_sq -- python3 $B > $O/pmc_sq.log 2>&1 || { tail -5 $O/pmc_sq.log; exit 1; }
python3 tools/pmc_kernels.py "$(find $O/pmc_sq -name '*counter_collection.csv' | head -n 1)" > $O/pmc_sq_summary.txt
grep -E "k_bias" $O/pmc_sq_summary.txt
echo "== $(date +%T) fetch"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 $B > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
echo "== $(date +%T) rate"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rate -- python3 tools/hub_rate.py --bias --calls 20 --out $O/hub_draws.json > $O/rate.log 2>&1 || { tail -5 $O/rate.log; exit 1; }
python3 tools/hub_rate.py --report $O/hub_draws.json --trace "$(find $O/rate -name '*kernel_trace.csv' | head -n 1)" --kernel k_bias_stream > $O/rate_report.txt 2>&1
tail -8 $O/rate_report.txt
echo "== $(date +%T) end"
