#!/bin/bash
# Round 4: kernel trace of one papers-like biased synchronous call (head with the LDS-staged
# stream kernel), and the same for products-like biased.
set -uo pipefail
N=${1:-r04o}
CALL_ARGS="--bias --scale 27 --ef 12 --dim 128" bash tools/r04_run.sh $N calltrace || exit $?
mv gpurun_out/$N/call_breakdown.txt gpurun_out/$N/call_breakdown_papers_bias.txt
rm -rf gpurun_out/$N/calls
CALL_ARGS="--bias" bash tools/r04_run.sh $N calltrace || exit $?
mv gpurun_out/$N/call_breakdown.txt gpurun_out/$N/call_breakdown_products_bias.txt
rm -rf gpurun_out/$N/calls
