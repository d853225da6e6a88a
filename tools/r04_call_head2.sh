#!/bin/bash
# Round 4 head check after the LDS-staged stream kernel: all GPU tests, smoke, the N = 2
# shared-device bench, N = 1 lines (default with the CPU baseline, biased, papers-like biased)
# and rocprof kernel stats of the default line.
set -uo pipefail
N=${1:-r04head2}
bash tools/r04_run.sh $N pytest smoke n2 bench bias papersbias rocprof
