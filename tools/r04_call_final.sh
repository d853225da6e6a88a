#!/bin/bash
# Round 4 final head check: every GPU test, smoke, the default bench line (with the CPU
# baseline), its rocprofv3 kernel stats, the biased lines and the N = 2 shared-device self-check.
set -uo pipefail
bash tools/r04_run.sh r04_final pytest smoke bench rocprof bias papersbias n2
