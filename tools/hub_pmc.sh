#!/bin/bash
# VALU counters of the uniform hub reservoir (and the other sampling kernels) in the sequential
# loop: one rocprofv3 --pmc pass (8 SQ counters), summarised by tools/pmc_kernels.py.
#   gpurun -- 'bash tools/hub_pmc.sh r01'
set -euo pipefail
R=${1:-r01}
O=gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_sq -- python3 bench.py --depth 1 --no-cpu-baseline --steps 50 --warmup 5 > $O/pmc_sq.log 2>&1
python3 tools/pmc_kernels.py "$(find $O/pmc_sq -name '*counter_collection.csv' | head -n 1)" > $O/pmc_sq_summary.txt
